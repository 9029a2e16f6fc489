// C++ tests of the drop-in layer, mirroring the reference's gtests (tests/*.cpp of lajoiepy/dpgo)
// plus the multi-robot example loop (examples/MultiRobotExample.cpp:175-264).  Needs a gfx950 GPU.
// Usage: test_dpgo <tests/golden dir>
#include <DPGO/DPGO_utils.h>
#include <DPGO/PGOAgent.h>
#include <DPGO/QuadraticOptimizer.h>
#include <DPGO/QuadraticProblem.h>
#include <DPGO/manifold/LiftedSEManifold.h>

#include <cmath>
#include <cstdio>
#include <fstream>
#include <functional>
#include <random>
#include <string>
#include <vector>

using namespace DPGO;

static int g_fail = 0;
#define EXPECT(cond)                                                        \
  do {                                                                      \
    if (!(cond)) {                                                          \
      std::printf("  FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond);       \
      ++g_fail;                                                             \
    }                                                                       \
  } while (0)

static Matrix rowmajor(long r, long c, std::initializer_list<double> v) {
  Matrix M(r, c);
  long k = 0;
  for (double x : v) {
    M(k / c, k % c) = x;
    ++k;
  }
  return M;
}

static Matrix randomMatrix(long r, long c, std::mt19937_64& rng) {
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  Matrix M(r, c);
  for (long j = 0; j < c; ++j)
    for (long i = 0; i < r; ++i) M(i, j) = U(rng);
  return M;
}

// tests/testTriangleGraph.cpp:7-65
static void testTriangleGraph() {
  unsigned id = 0, d = 3, r = 3;
  PGOAgentParameters options(d, r, 1);
  PGOAgent agent(id, options);
  Matrix Tw0 = Matrix::Identity(4, 4);
  Matrix Tw1 = rowmajor(4, 4, {0.1436, 0.7406, 0.6564, 1, -0.8179, -0.2845, 0.5000, 1, 0.5571, -0.6087, 0.5649, 1, 0, 0, 0, 1});
  Matrix Tw2 = rowmajor(4, 4, {-0.4069, -0.4150, -0.8138, 2, 0.4049, 0.7166, -0.5679, 2, 0.8188, -0.5606, -0.1236, 2, 0, 0, 0, 1});
  Matrix Ttrue(d, 3 * (d + 1));
  Ttrue.setBlock(0, 0, Tw0.block(0, 0, 3, 4));
  Ttrue.setBlock(0, 4, Tw1.block(0, 0, 3, 4));
  Ttrue.setBlock(0, 8, Tw2.block(0, 0, 3, 4));
  std::vector<RelativeSEMeasurement> odometry, private_lc, shared_lc;
  Matrix dT = Tw0.inverse() * Tw1;
  odometry.emplace_back(id, id, 0, 1, dT.block(0, 0, d, d), dT.block(0, d, d, 1), 1.0, 1.0);
  dT = Tw1.inverse() * Tw2;
  odometry.emplace_back(id, id, 1, 2, dT.block(0, 0, d, d), dT.block(0, d, d, 1), 1.0, 1.0);
  dT = Tw0.inverse() * Tw2;
  private_lc.emplace_back(id, id, 0, 2, dT.block(0, 0, d, d), dT.block(0, d, d, 1), 1.0, 1.0);
  agent.setPoseGraph(odometry, private_lc, shared_lc);
  Matrix Test;
  agent.getTrajectoryInLocalFrame(Test);
  EXPECT((Ttrue - Test).norm() <= 1e-4);
  agent.iterate();
  EXPECT(agent.getID() == id);
  EXPECT(agent.num_poses() == 3);
  EXPECT(agent.dimension() == d);
  EXPECT(agent.relaxation_rank() == r);
  agent.getTrajectoryInLocalFrame(Test);
  EXPECT((Ttrue - Test).norm() <= 1e-4);
  // the same graph, through localPoseGraphOptimization (r = d)
  Matrix Topt = agent.localPoseGraphOptimization();
  EXPECT(Topt.rows() == 3 && Topt.cols() == 12);
}

// tests/testLineGraph.cpp:7-31
static void testLineGraph() {
  unsigned id = 0, d = 3, r = 3;
  PGOAgentParameters options(d, r, 1);
  std::mt19937_64 rng(7);
  Matrix R = Matrix::Identity(d, d), t = randomMatrix(d, 1, rng);
  std::vector<RelativeSEMeasurement> odometry, private_lc, shared_lc;
  PGOAgent agent(id, options);
  for (unsigned i = 0; i < 4; ++i) odometry.emplace_back(id, id, i, i + 1, R, t, 1.0, 1.0);
  agent.setPoseGraph(odometry, private_lc, shared_lc);
  agent.iterate();
  EXPECT(agent.getID() == id);
  EXPECT(agent.num_poses() == 5);
  EXPECT(agent.dimension() == d);
  EXPECT(agent.relaxation_rank() == r);
}

// tests/testEigenMap.cpp:12-36: pose block j is the contiguous r*(d+1) doubles [Y_j | p_j]
static void testMemoryLayout() {
  const int d = 3, n = 10;
  Matrix X(d, (d + 1) * n);
  for (int i = 0; i < n; ++i) {
    X.setBlock(0, i * (d + 1), Matrix::Identity(d, d));
    for (int a = 0; a < d; ++a) X(a, i * (d + 1) + d) = 10.0 * i + a;
  }
  for (int i = 0; i < n; ++i) {
    const double* blk = X.data() + static_cast<size_t>(i) * d * (d + 1);
    for (int c = 0; c < d; ++c)
      for (int a = 0; a < d; ++a) EXPECT(blk[c * d + a] == (a == c ? 1.0 : 0.0));
    for (int a = 0; a < d; ++a) EXPECT(blk[d * d + a] == 10.0 * i + a);
  }
  // the device round trip preserves the layout: project() of points already on the manifold
  LiftedSEManifold M(d, d, n);
  EXPECT((M.project(X) - X).norm() <= 1e-12);
}

// tests/testUtils.cpp:12-53
static void testStiefel() {
  Matrix Y = fixedStiefelVariable(3, 5);
  EXPECT((Y.transpose() * Y - Matrix::Identity(3, 3)).norm() <= 1e-5);
  for (int i = 0; i < 10; ++i) EXPECT((fixedStiefelVariable(3, 5) - Y).norm() <= 1e-5);
  std::mt19937_64 rng(3);
  for (int j = 0; j < 50; ++j) {
    Matrix P = projectToStiefelManifold(randomMatrix(5, 3, rng));
    EXPECT((P.transpose() * P - Matrix::Identity(3, 3)).norm() <= 1e-5);
  }
  const int d = 3, r = 5, n = 100;
  LiftedSEManifold Manifold(r, d, n);
  Matrix X = Manifold.project(randomMatrix(r, (d + 1) * n, rng));
  EXPECT(X.rows() == r && X.cols() == (d + 1) * n);
  for (int i = 0; i < n; ++i) {
    Matrix Yi = X.block(0, i * (d + 1), r, d);
    EXPECT((Yi.transpose() * Yi - Matrix::Identity(d, d)).norm() <= 1e-5);
  }
}

// tests/testConstruction.cpp:7-19
static void testConstruction() {
  PGOAgentParameters options(3, 5, 1);
  PGOAgent agent(0, options);
  EXPECT(agent.getID() == 0);
  EXPECT(agent.num_poses() == 1);
  EXPECT(agent.dimension() == 3);
  EXPECT(agent.relaxation_rank() == 5);
}

static std::vector<RelativeSEMeasurement> read_meas_txt(const std::string& path, size_t& n) {
  std::ifstream in(path);
  std::vector<RelativeSEMeasurement> out;
  int d;
  size_t m;
  in >> d >> n >> m;
  for (size_t e = 0; e < m; ++e) {
    size_t p1, p2;
    in >> p1 >> p2;
    Matrix R(d, d), t(d, 1);
    for (int u = 0; u < d; ++u)
      for (int v = 0; v < d; ++v) in >> R(u, v);
    for (int u = 0; u < d; ++u) in >> t(u, 0);
    double k, ta;
    in >> k >> ta;
    out.emplace_back(0, 0, p1, p2, R, t, k, ta);
  }
  return out;
}

static Matrix read_matrix_txt(const std::string& path) {
  std::ifstream in(path);
  long r, c;
  in >> r >> c;
  Matrix M(r, c);
  for (long i = 0; i < r; ++i)
    for (long j = 0; j < c; ++j) in >> M(i, j);
  return M;
}

// examples/MultiRobotExample.cpp:21-282 (5 robots, r = 5, acceleration, reference defaults),
// starting from the oracle's chordal initialisation; prints one line per iteration.
static void multiRobotExample(const std::string& golden) {
  size_t n = 0;
  auto dataset = read_meas_txt(golden + "/smallGrid3D.meas.txt", n);
  const Matrix X0 = read_matrix_txt(golden + "/smallGrid3D.X0.txt");
  const unsigned d = 3, r = 5, num_robots = 5, numIters = 30;
  QuadraticProblem problemCentral(n, d, r);
  problemCentral.setQ(constructConnectionLaplacianSE(dataset, n));
  const unsigned per = static_cast<unsigned>(n / num_robots);
  auto range = [&](unsigned robot, unsigned& s, unsigned& e) {
    s = robot * per;
    e = robot == num_robots - 1 ? static_cast<unsigned>(n) : (robot + 1) * per;
  };
  std::vector<std::pair<unsigned, unsigned>> PoseMap(n);
  for (unsigned robot = 0; robot < num_robots; ++robot) {
    unsigned s, e;
    range(robot, s, e);
    for (unsigned i = s; i < e; ++i) PoseMap[i] = {robot, i - s};
  }
  std::vector<std::vector<RelativeSEMeasurement>> odo(num_robots), priv(num_robots), shared(num_robots);
  for (const auto& mIn : dataset) {
    const auto src = PoseMap[mIn.p1], dst = PoseMap[mIn.p2];
    RelativeSEMeasurement m(src.first, dst.first, src.second, dst.second, mIn.R, mIn.t, mIn.kappa, mIn.tau);
    if (src.first == dst.first) {
      (src.second + 1 == dst.second ? odo : priv)[src.first].push_back(m);
    } else {
      shared[src.first].push_back(m);
      shared[dst.first].push_back(m);
    }
  }
  std::vector<std::unique_ptr<PGOAgent>> agents;
  for (unsigned robot = 0; robot < num_robots; ++robot) {
    PGOAgentParameters options(d, r, num_robots);
    options.acceleration = true;
    agents.emplace_back(new PGOAgent(robot, options));
    if (robot > 0) {
      Matrix M;
      agents[0]->getLiftingMatrix(M);
      agents[robot]->setLiftingMatrix(M);
    }
    agents[robot]->setPoseGraph(odo[robot], priv[robot], shared[robot]);
  }
  for (unsigned robot = 0; robot < num_robots; ++robot) {
    unsigned s, e;
    range(robot, s, e);
    agents[robot]->setX(X0.block(0, s * (d + 1), r, (e - s) * (d + 1)));
  }
  Matrix Xopt(r, static_cast<long>(n * (d + 1)));
  unsigned selected = 0;
  const double cost0 = 2 * problemCentral.f(X0);
  double cost = cost0, best = cost0;
  for (unsigned iter = 0; iter < numIters; ++iter) {
    PGOAgent* sel = agents[selected].get();
    for (auto& a : agents)
      if (a->getID() != selected) a->iterate(false);
    for (auto& a : agents) {
      if (a->getID() == selected) continue;
      PoseDict pd;
      if (!a->getSharedPoseDict(pd)) continue;
      sel->setNeighborStatus(a->getStatus());
      sel->updateNeighborPoses(a->getID(), pd);
    }
    for (auto& a : agents) {
      if (a->getID() == selected) continue;
      PoseDict pd;
      if (!a->getAuxSharedPoseDict(pd)) continue;
      sel->setNeighborStatus(a->getStatus());
      sel->updateAuxNeighborPoses(a->getID(), pd);
    }
    sel->iterate(true);
    for (unsigned robot = 0; robot < num_robots; ++robot) {
      unsigned s, e;
      range(robot, s, e);
      Matrix Xr;
      agents[robot]->getX(Xr);
      Xopt.setBlock(0, s * (d + 1), Xr);
    }
    const Matrix RG = problemCentral.RieGrad(Xopt);
    const double gn = RG.norm();
    cost = 2 * problemCentral.f(Xopt);
    best = std::min(best, cost);
    std::printf("ITER %u %u %.17g %.17g\n", iter, selected, cost, gn);
    if (gn < 0.1) break;
    std::vector<double> norms;
    for (unsigned robot = 0; robot < num_robots; ++robot) {
      unsigned s, e;
      range(robot, s, e);
      norms.push_back(RG.block(0, s * (d + 1), r, (e - s) * (d + 1)).norm());
    }
    selected = static_cast<unsigned>(std::max_element(norms.begin(), norms.end()) - norms.begin());
  }
  EXPECT(best < 0.7 * cost0);  // (the GNC_TLS re-weighting at iteration 29 raises the unweighted cost)
}

int main(int argc, char** argv) {
  const std::string golden = argc > 1 ? argv[1] : "tests/golden";
  struct T {
    const char* name;
    std::function<void()> fn;
  } tests[] = {{"Construction", testConstruction},
               {"MemoryLayout", testMemoryLayout},
               {"Stiefel", testStiefel},
               {"TriangleGraph", testTriangleGraph},
               {"LineGraph", testLineGraph},
               {"MultiRobotExample", [&] { multiRobotExample(golden); }}};
  for (auto& t : tests) {
    const int before = g_fail;
    try {
      t.fn();
    } catch (const std::exception& e) {
      std::printf("  EXCEPTION %s\n", e.what());
      ++g_fail;
    }
    std::printf("[%s] %s\n", g_fail == before ? "PASS" : "FAIL", t.name);
  }
  std::printf("%s\n", g_fail ? "SOME TESTS FAILED" : "ALL TESTS PASSED");
  return g_fail ? 1 : 0;
}

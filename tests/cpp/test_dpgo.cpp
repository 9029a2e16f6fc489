// C++ tests of the drop-in layer, mirroring the reference's gtests (tests/*.cpp of lajoiepy/dpgo)
// plus the multi-robot example loop (examples/MultiRobotExample.cpp:175-264).  Needs a gfx950 GPU.
// Usage: test_dpgo <tests/golden dir> [--host]   (--host: only the cases that make no GPU call)
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

// Eigen::Quaterniond::UnitRandom().toRotationMatrix() restated: normalised 4-D Gaussian quaternion
static Matrix randomRotation(std::mt19937_64& rng) {
  std::normal_distribution<double> N(0.0, 1.0);
  double q[4], nn = 0;
  for (double& x : q) {
    x = N(rng);
    nn += x * x;
  }
  nn = std::sqrt(nn);
  const double w = q[0] / nn, x = q[1] / nn, y = q[2] / nn, z = q[3] / nn;
  return rowmajor(3, 3, {1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                         2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                         2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)});
}

static Vector constVec(size_t n, double v) {
  Vector o(static_cast<long>(n), 1);
  for (size_t i = 0; i < n; ++i) o(static_cast<long>(i), 0) = v;
  return o;
}

// tests/testUtils.cpp:55-72 (plus the tabulated quantiles chi2inv(0.95, 4), chi2inv(0.9, 6))
static void testChi2Inv() {
  EXPECT(std::fabs(chi2inv(0.95, 4) - 9.487729036781154) <= 1e-9);
  EXPECT(std::fabs(chi2inv(0.9, 6) - 10.64464067566842) <= 1e-9);
  EXPECT(std::fabs(chi2inv(0.5, 2) - 2 * std::log(2.0)) <= 1e-12);
  const double threshold = chi2inv(0.95, 4);
  std::mt19937 rng(7);
  std::chi_squared_distribution<double> dist(4);
  int count = 0;
  for (int i = 0; i < 100000; ++i) count += dist(rng) < threshold;
  EXPECT(std::fabs(count / 100000.0 - 0.95) <= 0.01);
}

// tests/testUtils.cpp:74-118
static void testRobustSingleRotationAveraging() {
  std::mt19937_64 rng(11);
  for (int trial = 0; trial < 50; ++trial) {
    const Matrix RTrue = randomRotation(rng);
    Matrix ROpt;
    std::vector<size_t> inl;
    robustSingleRotationAveraging(ROpt, inl, {RTrue}, constVec(1, 1.0), angular2ChordalSO3(0.5));
    EXPECT((ROpt - RTrue).norm() <= 1e-8);
    EXPECT(inl.size() == 1 && inl[0] == 0);
  }
  for (int trial = 0; trial < 50; ++trial) {
    const double tol = angular2ChordalSO3(0.02), cbar = angular2ChordalSO3(0.3);
    const Matrix RTrue = randomRotation(rng);
    std::vector<Matrix> RVec(10, RTrue);
    while (RVec.size() < 50) {
      Matrix RRand = randomRotation(rng);
      if ((RRand - RTrue).norm() > 1.2 * cbar) RVec.push_back(RRand);
    }
    Matrix ROpt;
    std::vector<size_t> inl;
    robustSingleRotationAveraging(ROpt, inl, RVec, constVec(50, 1.0), cbar);
    EXPECT(std::fabs(ROpt.determinant() - 1.0) < 1e-8);
    EXPECT((ROpt - RTrue).norm() <= tol);
    EXPECT(inl.size() == 10);
    for (size_t i = 0; i < inl.size() && i < 10; ++i) EXPECT(inl[i] == i);
  }
}

// tests/testUtils.cpp:120-190
static void testRobustSinglePoseAveraging() {
  std::mt19937_64 rng(12);
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  const double barc = RobustCost::computeErrorThresholdAtQuantile(0.9, 3);
  for (int trial = 0; trial < 50; ++trial) {
    const Matrix RTrue = randomRotation(rng);
    const Vector tTrue = Matrix::Zero(3, 1);
    Matrix ROpt;
    Vector tOpt;
    std::vector<size_t> inl;
    robustSinglePoseAveraging(ROpt, tOpt, inl, {RTrue}, {tTrue}, constVec(1, 10000), constVec(1, 100), barc);
    EXPECT((ROpt - RTrue).norm() <= 1e-8);
    EXPECT((tOpt - tTrue).norm() <= 1e-8);
    EXPECT(inl.size() == 1 && inl[0] == 0);
  }
  for (int trial = 0; trial < 50; ++trial) {
    const double kappa = 10000, tau = 100;
    const Matrix RTrue = randomRotation(rng);
    const Vector tTrue = Matrix::Zero(3, 1);
    std::vector<Matrix> RVec(10, RTrue);
    std::vector<Vector> tVec(10, tTrue);
    while (RVec.size() < 50) {
      Matrix RRand = randomRotation(rng);
      Vector tRand(3, 1);
      for (long i = 0; i < 3; ++i) tRand(i, 0) = U(rng);
      const double rSq = kappa * (RTrue - RRand).squaredNorm() + tau * (tTrue - tRand).squaredNorm();
      if (std::sqrt(rSq) > 1.2 * barc) {
        RVec.push_back(RRand);
        tVec.push_back(tRand);
      }
    }
    Matrix ROpt;
    Vector tOpt;
    std::vector<size_t> inl;
    robustSinglePoseAveraging(ROpt, tOpt, inl, RVec, tVec, constVec(50, kappa), constVec(50, tau), barc);
    EXPECT((ROpt - RTrue).norm() <= angular2ChordalSO3(0.02));
    EXPECT((tOpt - tTrue).norm() <= 1e-2);
    EXPECT(inl.size() == 10);
    for (size_t i = 0; i < inl.size() && i < 10; ++i) EXPECT(inl[i] == i);
  }
}

// PGOAgent::initializeInGlobalFrame (src/PGOAgent.cpp:250-432) on a noise-free 3D lattice split over
// two robots: robot 1 starts in the frame of its own first pose (chordal local init); after
// receiving robot 0's public poses it must hold the ground truth in robot 0's frame.  Two shared
// loop closures are corrupted and must be rejected by the robust rotation average.
static void testMultiRobotInitialization() {
  const unsigned d = 3, r = 5, k = 4, n = k * k * k, half = n / 2;
  std::mt19937_64 rng(21);
  std::vector<Matrix> Rw(n), tw(n);
  for (unsigned i = 0; i < n; ++i) {
    Rw[i] = randomRotation(rng);
    tw[i] = rowmajor(3, 1, {double(i % k), double((i / k) % k), double(i / (k * k))});
  }
  auto meas = [&](unsigned a, unsigned b) {
    RelativeSEMeasurement m;
    m.r1 = a < half ? 0 : 1;
    m.r2 = b < half ? 0 : 1;
    m.p1 = a < half ? a : a - half;
    m.p2 = b < half ? b : b - half;
    m.R = Rw[a].transpose() * Rw[b];
    m.t = Rw[a].transpose() * (tw[b] - tw[a]);
    m.kappa = 12.5;
    m.tau = 100;
    return m;
  };
  std::vector<RelativeSEMeasurement> odo[2], priv[2], shared[2];
  int corrupted = 0;
  for (unsigned a = 0; a < n; ++a)
    for (unsigned b = a + 1; b < n; ++b) {
      const double dist = (tw[b] - tw[a]).norm();
      if (b != a + 1 && dist > 1.0 + 1e-9) continue;  // odometry chain + lattice neighbours
      RelativeSEMeasurement m = meas(a, b);
      if (m.r1 == m.r2) {
        (b == a + 1 ? odo : priv)[m.r1].push_back(m);
      } else {
        if (corrupted < 2 && (a % 7) == 3) {
          m.R = randomRotation(rng);  // outlier inter-robot loop closure
          ++corrupted;
        }
        shared[0].push_back(m);
        shared[1].push_back(m);
      }
    }
  PGOAgentParameters opts(d, r, 2);
  opts.robustCostType = L2;
  PGOAgent a0(0, opts), a1(1, opts);
  a0.setPoseGraph(odo[0], priv[0], shared[0]);
  a1.setPoseGraph(odo[1], priv[1], shared[1]);
  Matrix YLift;
  EXPECT(a0.getLiftingMatrix(YLift));
  a1.setLiftingMatrix(YLift);
  EXPECT(a0.getState() == INITIALIZED);
  EXPECT(a1.getState() == WAIT_FOR_INITIALIZATION);
  PoseDict dict;
  EXPECT(a0.getSharedPoseDict(dict));
  EXPECT(!dict.empty());
  a1.setNeighborStatus(a0.getStatus());
  Matrix Tr;
  {  // per-public-pose transforms vs the true T_world0_frame1 (robot 1's frame = its first pose)
    Matrix Ttrue = Matrix::Identity(4, 4);
    Ttrue.setBlock(0, 0, Rw[0].transpose() * Rw[half]);
    Ttrue.setBlock(0, 3, Rw[0].transpose() * (tw[half] - tw[0]));
    std::vector<Matrix> RV;
    std::vector<size_t> exact;
    for (const auto& kv : dict) {
      const Matrix T = a1.computeNeighborTransform(kv.first, kv.second);
      if ((T - Ttrue).norm() <= 1e-12) exact.push_back(RV.size());
      RV.push_back(T.block(0, 0, 3, 3));
    }
    EXPECT(exact.size() + 2 == dict.size());  // the two corrupted closures
    Matrix Ro;
    std::vector<size_t> inl;
    robustSingleRotationAveraging(Ro, inl, RV, Vector(), angular2ChordalSO3(0.5));
    EXPECT(inl == exact);
    // GNC returns the average solved with the last-but-one weights (src/DPGO_utils.cpp:618-637), so
    // the outliers keep a small weight in ROpt: the reference's tolerance (testUtils.cpp:95)
    Tr = a1.computeRobustNeighborTransformTwoStage(0, dict);
    EXPECT((Tr.block(0, 0, 3, 3) - Ttrue.block(0, 0, 3, 3)).norm() <= angular2ChordalSO3(0.02));
    EXPECT((Tr.block(0, 0, 3, 3) - Ro).norm() <= 1e-14);
  }
  a1.updateNeighborPoses(0, dict);
  EXPECT(a1.getState() == INITIALIZED);
  Matrix X1;
  a1.getX(X1);
  const Matrix T1 = YLift.transpose() * X1;
  // X1 = YLift * (Tr * T_local): robot 1's local chordal init is the ground truth in the frame of its
  // first pose, so T1 = Tr * (T_frame1_i) exactly; and within the averaging tolerance of the truth
  double err = 0, dev = 0;
  Matrix Tf1 = Matrix::Identity(4, 4);
  for (unsigned i = 0; i < n - half; ++i) {
    Tf1.setBlock(0, 0, Rw[half].transpose() * Rw[half + i]);
    Tf1.setBlock(0, 3, Rw[half].transpose() * (tw[half + i] - tw[half]));
    const Matrix Ti = (Tr * Tf1).block(0, 0, 3, 4);
    err = std::max(err, (T1.block(0, i * (d + 1), d, d + 1) - Ti).norm());
    const Matrix R = Rw[0].transpose() * Rw[half + i];
    const Matrix t = Rw[0].transpose() * (tw[half + i] - tw[0]);
    dev = std::max(dev, (T1.block(0, i * (d + 1), d, d) - R).norm());
    dev = std::max(dev, (T1.block(0, i * (d + 1) + d, d, 1) - t).norm() / 10.0);
  }
  EXPECT(corrupted == 2);
  EXPECT(err <= 1e-10);
  EXPECT(dev <= angular2ChordalSO3(0.02));
  if (err > 1e-10 || dev > angular2ChordalSO3(0.02)) std::printf("  pose error %.3e, vs truth %.3e\n", err, dev);
}

int main(int argc, char** argv) {
  const std::string golden = argc > 1 ? argv[1] : "tests/golden";
  const bool host_only = argc > 2 && std::string(argv[2]) == "--host";
  struct T {
    const char* name;
    std::function<void()> fn;
    bool host;
  } tests[] = {{"Chi2Inv", testChi2Inv, true},
               {"RobustSingleRotationAveraging", testRobustSingleRotationAveraging, true},
               {"RobustSinglePoseAveraging", testRobustSinglePoseAveraging, true},
               {"MultiRobotInitialization", testMultiRobotInitialization, false},
               {"Construction", testConstruction, true},
               {"MemoryLayout", testMemoryLayout},
               {"Stiefel", testStiefel},
               {"TriangleGraph", testTriangleGraph},
               {"LineGraph", testLineGraph},
               {"MultiRobotExample", [&] { multiRobotExample(golden); }}};
  for (auto& t : tests) {
    if (host_only && !t.host) continue;
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

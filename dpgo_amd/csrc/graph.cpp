// Pose-graph inputs on the host: g2o reader, synthetic 3D grid, connection Laplacian (BSR),
// odometry initialisation and grid partitioning.  See include/dpgo_rbcd.h.
//
// The grid generator must produce bit-identical graphs to oracle/dpgo_oracle.py::grid3d, so
// floating-point contraction is disabled and every expression keeps the oracle's order.
#pragma clang fp contract(off)

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <set>
#include <sstream>
#include <string>
#include <utility>
#include <vector>

#include "graph_internal.h"

using namespace dpgo;

namespace {

struct SplitMix64 {
  uint64_t state;
  bool has = false;
  double cached = 0.0;
  explicit SplitMix64(uint64_t s) : state(s) {}
  uint64_t next() {
    state += 0x9E3779B97F4A7C15ULL;
    uint64_t z = state;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
  }
  double uniform() { return static_cast<double>(next() >> 11) * (1.0 / 9007199254740992.0); }
  double normal() {
    if (has) {
      has = false;
      return cached;
    }
    const double u1 = 1.0 - uniform();
    const double u2 = uniform();
    const double rad = std::sqrt(-2.0 * std::log(u1));
    const double ang = 6.283185307179586 * u2;
    cached = rad * std::sin(ang);
    has = true;
    return rad * std::cos(ang);
  }
};

typedef double M3[3][3];

void mm3(const M3 A, const M3 B, M3 C) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) C[i][j] = A[i][0] * B[0][j] + A[i][1] * B[1][j] + A[i][2] * B[2][j];
}

void quat_rot(const double q[4], M3 R) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  const double nrm = std::sqrt(w * w + x * x + y * y + z * z);
  w = w / nrm;
  x = x / nrm;
  y = y / nrm;
  z = z / nrm;
  R[0][0] = 1 - 2 * (y * y + z * z);
  R[0][1] = 2 * (x * y - z * w);
  R[0][2] = 2 * (x * z + y * w);
  R[1][0] = 2 * (x * y + z * w);
  R[1][1] = 1 - 2 * (x * x + z * z);
  R[1][2] = 2 * (y * z - x * w);
  R[2][0] = 2 * (x * z - y * w);
  R[2][1] = 2 * (y * z + x * w);
  R[2][2] = 1 - 2 * (x * x + y * y);
}

void rodrigues(const double w[3], M3 R) {
  const double wx = w[0], wy = w[1], wz = w[2];
  const double th2 = wx * wx + wy * wy + wz * wz;
  const double th = std::sqrt(th2);
  const double K[3][3] = {{0.0, -wz, wy}, {wz, 0.0, -wx}, {-wy, wx, 0.0}};
  double A, B;
  if (th < 1e-12) {
    A = 1.0;
    B = 0.5;
  } else {
    A = std::sin(th) / th;
    B = (1.0 - std::cos(th)) / th2;
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      const double kk = K[i][0] * K[0][j] + K[i][1] * K[1][j] + K[i][2] * K[2][j];
      R[i][j] = (i == j ? 1.0 : 0.0) + A * K[i][j] + B * kk;
    }
}

// Eigen::Quaterniond(w,x,y,z).toRotationMatrix(), no normalisation (src/DPGO_utils.cpp:169)
void quat_to_rot_eigen(double qw, double qx, double qy, double qz, double* R) {
  const double tx = 2.0 * qx, ty = 2.0 * qy, tz = 2.0 * qz;
  const double twx = tx * qw, twy = ty * qw, twz = tz * qw;
  const double txx = tx * qx, txy = ty * qx, txz = tz * qx;
  const double tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
  const double v[9] = {1.0 - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1.0 - (txx + tzz),
                       tyz - twx, txz - twy, tyz + twx, 1.0 - (txx + tyy)};
  std::memcpy(R, v, sizeof(v));
}

// trace(M^-1) with Eigen's fixed-size closed-form inverses (the reader calls
// TranCov.inverse().trace(), src/DPGO_utils.cpp:131,178,185): invdet = 1/det, r_ii = cof_ii * invdet.
bool inv_trace_2(double a, double b, double d, double* tr) {
  const double det = a * d - b * b;
  if (det == 0.0) return false;
  const double invdet = 1.0 / det;
  *tr = d * invdet + a * invdet;
  return true;
}

bool inv_trace_3(const double m[3][3], double* tr) {
  const double c00 = m[1][1] * m[2][2] - m[1][2] * m[2][1];
  const double c10 = m[2][1] * m[0][2] - m[2][2] * m[0][1];
  const double c20 = m[0][1] * m[1][2] - m[0][2] * m[1][1];
  const double det = c00 * m[0][0] + c10 * m[1][0] + c20 * m[2][0];
  if (det == 0.0) return false;
  const double invdet = 1.0 / det;
  const double c11 = m[2][2] * m[0][0] - m[2][0] * m[0][2];
  const double c22 = m[0][0] * m[1][1] - m[0][1] * m[1][0];
  *tr = c00 * invdet + c11 * invdet + c22 * invdet;
  return true;
}

void finish(dpgo_graph g) {
  int n = 0;
  std::set<std::pair<int, int>> seen;
  g->duplicates = 0;
  for (size_t e = 0; e < g->p1.size(); ++e) {
    n = std::max(n, std::max(g->p1[e], g->p2[e]) + 1);
    if (!seen.insert({g->p1[e], g->p2[e]}).second) ++g->duplicates;
  }
  g->n = n;
}

}  // namespace

namespace dpgo {

// Per-edge Q blocks (a3): Q_ii += T Om T^T, Q_jj += Om, Q_ij = -T Om, Q_ji = -Om T^T.
// Blocks are produced in the device convention: block (row, col) column-major.
void edge_blocks(int d, const double* R, const double* t, double kappa, double tau, double w, double* Wii,
                 double* Wjj, double* Wij, double* Wji) {
  const int b = d + 1;
  double T[4][4] = {{0}}, Om[4] = {0};
  for (int u = 0; u < d; ++u) {
    for (int v = 0; v < d; ++v) T[u][v] = R[u * d + v];
    T[u][d] = t[u];
    Om[u] = w * kappa;
  }
  T[d][d] = 1.0;
  Om[d] = w * tau;
  for (int u = 0; u < b; ++u)
    for (int v = 0; v < b; ++v) {
      double s = 0.0;
      for (int q = 0; q < b; ++q) s += T[u][q] * Om[q] * T[v][q];
      Wii[v * b + u] = s;                           // (T Om T^T)(u,v)
      Wjj[v * b + u] = (u == v) ? Om[u] : 0.0;      // Om
      Wij[v * b + u] = -T[u][v] * Om[v];            // -(T Om)(u,v)
      Wji[v * b + u] = -Om[u] * T[v][u];            // -(Om T^T)(u,v)
    }
}

void BsrBuilder::freeze() {
  out.rowptr.assign(n + 1, 0);
  for (int j = 0; j < n; ++j) {
    auto& c = cols[j];
    std::sort(c.begin(), c.end());
    c.erase(std::unique(c.begin(), c.end()), c.end());
    out.rowptr[j + 1] = out.rowptr[j] + static_cast<int>(c.size());
  }
  out.col.resize(out.rowptr[n]);
  for (int j = 0; j < n; ++j) std::copy(cols[j].begin(), cols[j].end(), out.col.begin() + out.rowptr[j]);
  out.blocks.assign(static_cast<size_t>(out.rowptr[n]) * b * b, 0.0);
  std::vector<std::vector<int>>().swap(cols);
}

double* BsrBuilder::block(int i, int j) {
  for (int k = out.rowptr[i]; k < out.rowptr[i + 1]; ++k)
    if (out.col[k] == j) return &out.blocks[static_cast<size_t>(k) * b * b];
  return nullptr;
}

void BsrBuilder::add(int i, int j, const double* blk) {
  double* dst = block(i, j);
  for (int q = 0; q < b * b; ++q) dst[q] += blk[q];
}

}  // namespace dpgo

extern "C" {

int dpgo_graph_read_g2o(const char* path, dpgo_graph* out) {
  if (!out || !path) return fail(DPGO_HIP_EINVAL, "null argument");
  std::ifstream in(path);
  if (!in) return fail(DPGO_HIP_EINVAL, std::string("cannot open ") + path);
  auto* g = new dpgo_graph_s();
  std::string line, tok;
  while (std::getline(in, line)) {
    std::istringstream ss(line);
    if (!(ss >> tok)) continue;  // blank line: skipped (App. B2 fix)
    unsigned long long ki, kj;
    if (tok == "EDGE_SE2") {
      double dx, dy, th, I11, I12, I13, I22, I23, I33;
      if (!(ss >> ki >> kj >> dx >> dy >> th >> I11 >> I12 >> I13 >> I22 >> I23 >> I33)) continue;
      if (g->d == 0) g->d = 2;
      if (g->d != 2) {
        delete g;
        return fail(DPGO_HIP_EINVAL, "mixed 2D/3D edges");
      }
      const double c = std::cos(th), s = std::sin(th);
      const double Rv[4] = {c, -s, s, c};
      g->R.insert(g->R.end(), Rv, Rv + 4);
      g->t.push_back(dx);
      g->t.push_back(dy);
      double tr;
      if (!inv_trace_2(I11, I12, I22, &tr)) tr = INFINITY;
      g->tau.push_back(2.0 / tr);   // :129-131
      g->kappa.push_back(I33);      // :133
      (void)I13;
      (void)I23;
    } else if (tok == "EDGE_SE3:QUAT") {
      double v[7], I[21];
      if (!(ss >> ki >> kj)) continue;
      bool ok = true;
      for (double& x : v) ok = ok && static_cast<bool>(ss >> x);
      for (double& x : I) ok = ok && static_cast<bool>(ss >> x);
      if (!ok) continue;
      if (g->d == 0) g->d = 3;
      if (g->d != 3) {
        delete g;
        return fail(DPGO_HIP_EINVAL, "mixed 2D/3D edges");
      }
      double Rm[9];
      quat_to_rot_eigen(v[6], v[3], v[4], v[5], Rm);
      g->R.insert(g->R.end(), Rm, Rm + 9);
      g->t.insert(g->t.end(), v, v + 3);
      const double Tc[3][3] = {{I[0], I[1], I[2]}, {I[1], I[6], I[7]}, {I[2], I[7], I[11]}};
      const double Rc[3][3] = {{I[15], I[16], I[17]}, {I[16], I[18], I[19]}, {I[17], I[19], I[20]}};
      double tt, tr;
      if (!inv_trace_3(Tc, &tt)) tt = INFINITY;
      if (!inv_trace_3(Rc, &tr)) tr = INFINITY;
      g->tau.push_back(3.0 / tt);           // :176-178
      g->kappa.push_back(3.0 / (2.0 * tr)); // :183-185
    } else {
      continue;  // VERTEX_* / FIX / unknown tokens ignored (App. B2)
    }
    // GTSAM key -> (robot char, 48-bit index) (src/DPGO_utils.cpp:21-33)
    g->r1.push_back(static_cast<int>((ki >> 56) & 0xFF));
    g->r2.push_back(static_cast<int>((kj >> 56) & 0xFF));
    g->p1.push_back(static_cast<int>(ki & ((1ULL << 48) - 1)));
    g->p2.push_back(static_cast<int>(kj & ((1ULL << 48) - 1)));
  }
  finish(g);
  *out = g;
  return DPGO_HIP_OK;
}

int dpgo_graph_from_arrays(int d, int n, int m, const int* p1, const int* p2, const double* R, const double* t,
                           const double* kappa, const double* tau, dpgo_graph* out) {
  if (!out || (d != 2 && d != 3) || m < 0) return fail(DPGO_HIP_EINVAL, "bad graph arrays");
  auto* g = new dpgo_graph_s();
  g->d = d;
  g->p1.assign(p1, p1 + m);
  g->p2.assign(p2, p2 + m);
  g->r1.assign(m, 0);
  g->r2.assign(m, 0);
  g->R.assign(R, R + static_cast<size_t>(m) * d * d);
  g->t.assign(t, t + static_cast<size_t>(m) * d);
  g->kappa.assign(kappa, kappa + m);
  g->tau.assign(tau, tau + m);
  finish(g);
  if (n > g->n) g->n = n;
  *out = g;
  return DPGO_HIP_OK;
}

int dpgo_graph_grid3d(int k, unsigned long long seed, double rot_sigma, double trans_sigma, dpgo_graph* out) {
  if (!out || k < 2 || k > 200) return fail(DPGO_HIP_EINVAL, "grid side must be in [2, 200]");
  auto* g = new dpgo_graph_s();
  g->d = 3;
  const int n = k * k * k, kk = k * k;
  g->coords.resize(static_cast<size_t>(n) * 3);
  std::vector<int> lut(n);
  for (int i = 0; i < n; ++i) {
    const int z = i / kk;
    int idx = i % kk;
    if (z & 1) idx = kk - 1 - idx;
    const int yy = idx / k;
    int xx = idx % k;
    if (yy & 1) xx = k - 1 - xx;
    g->coords[3 * i] = xx;
    g->coords[3 * i + 1] = yy;
    g->coords[3 * i + 2] = z;
    lut[xx + k * (yy + k * z)] = i;
  }
  // edges: all axis-aligned lattice-neighbour pairs (low, high), sorted by (low, high)
  std::vector<std::pair<int, int>> edges;
  edges.reserve(static_cast<size_t>(3) * kk * (k - 1));
  for (int i = 0; i < n; ++i) {
    const int x = g->coords[3 * i], y = g->coords[3 * i + 1], z = g->coords[3 * i + 2];
    const int nb[6][3] = {{x - 1, y, z}, {x + 1, y, z}, {x, y - 1, z}, {x, y + 1, z}, {x, y, z - 1}, {x, y, z + 1}};
    std::vector<int> hi;
    for (auto& c : nb) {
      if (c[0] < 0 || c[0] >= k || c[1] < 0 || c[1] >= k || c[2] < 0 || c[2] >= k) continue;
      const int j = lut[c[0] + k * (c[1] + k * c[2])];
      if (j > i) hi.push_back(j);
    }
    std::sort(hi.begin(), hi.end());
    for (int j : hi) edges.emplace_back(i, j);
  }
  SplitMix64 rng(seed);
  std::vector<double> Rgt(static_cast<size_t>(n) * 9);
  for (int i = 0; i < n; ++i) {
    double q[4];
    for (double& x : q) x = rng.normal();
    M3 Ri;
    quat_rot(q, Ri);
    for (int u = 0; u < 3; ++u)
      for (int v = 0; v < 3; ++v) Rgt[9 * static_cast<size_t>(i) + 3 * u + v] = Ri[u][v];
  }
  const size_t m = edges.size();
  g->p1.resize(m);
  g->p2.resize(m);
  g->r1.assign(m, 0);
  g->r2.assign(m, 0);
  g->R.resize(m * 9);
  g->t.resize(m * 3);
  g->kappa.assign(m, 12.5);
  g->tau.assign(m, 100.0);
  for (size_t e = 0; e < m; ++e) {
    const int i = edges[e].first, j = edges[e].second;
    M3 RiT, Rj, A, E, Rij;
    for (int u = 0; u < 3; ++u)
      for (int v = 0; v < 3; ++v) {
        RiT[u][v] = Rgt[9 * static_cast<size_t>(i) + 3 * v + u];
        Rj[u][v] = Rgt[9 * static_cast<size_t>(j) + 3 * u + v];
      }
    double eps[3], nz[3];
    for (double& x : eps) x = rot_sigma * rng.normal();
    for (double& x : nz) x = trans_sigma * rng.normal();
    mm3(RiT, Rj, A);
    rodrigues(eps, E);
    mm3(A, E, Rij);
    double dt[3];
    for (int c = 0; c < 3; ++c)
      dt[c] = static_cast<double>(g->coords[3 * static_cast<size_t>(j) + c] - g->coords[3 * static_cast<size_t>(i) + c]);
    g->p1[e] = i;
    g->p2[e] = j;
    for (int u = 0; u < 3; ++u) {
      for (int v = 0; v < 3; ++v) g->R[9 * e + 3 * u + v] = Rij[u][v];
      g->t[3 * e + u] = RiT[u][0] * dt[0] + RiT[u][1] * dt[1] + RiT[u][2] * dt[2] + nz[u];
    }
  }
  finish(g);
  *out = g;
  return DPGO_HIP_OK;
}

int dpgo_graph_info(dpgo_graph g, int* d, int* n, int* m, int* duplicates) {
  if (!g) return fail(DPGO_HIP_EINVAL, "null graph");
  if (d) *d = g->d;
  if (n) *n = g->n;
  if (m) *m = static_cast<int>(g->p1.size());
  if (duplicates) *duplicates = g->duplicates;
  return DPGO_HIP_OK;
}

int dpgo_graph_copy_out(dpgo_graph g, int* p1, int* p2, double* R, double* t, double* kappa, double* tau) {
  if (!g) return fail(DPGO_HIP_EINVAL, "null graph");
  const size_t m = g->p1.size();
  if (p1) std::copy(g->p1.begin(), g->p1.end(), p1);
  if (p2) std::copy(g->p2.begin(), g->p2.end(), p2);
  if (R) std::copy(g->R.begin(), g->R.end(), R);
  if (t) std::copy(g->t.begin(), g->t.end(), t);
  if (kappa) std::copy(g->kappa.begin(), g->kappa.end(), kappa);
  if (tau) std::copy(g->tau.begin(), g->tau.end(), tau);
  (void)m;
  return DPGO_HIP_OK;
}

int dpgo_graph_destroy(dpgo_graph g) {
  delete g;
  return DPGO_HIP_OK;
}

int dpgo_graph_laplacian_bsr(dpgo_graph g, long long* nnzb, int* browptr, int* bcol, double* blocks) {
  if (!g || !nnzb) return fail(DPGO_HIP_EINVAL, "null argument");
  const int d = g->d, b = d + 1;
  if (!g->q_cache_valid) {
    BsrBuilder B(g->n, b);
    for (size_t e = 0; e < g->p1.size(); ++e) {
      B.touch(g->p1[e], g->p2[e]);
      B.touch(g->p2[e], g->p1[e]);
    }
    B.freeze();
    double Wii[16], Wjj[16], Wij[16], Wji[16];
    for (size_t e = 0; e < g->p1.size(); ++e) {
      const int i = g->p1[e], j = g->p2[e];
      edge_blocks(d, &g->R[e * d * d], &g->t[e * d], g->kappa[e], g->tau[e], 1.0, Wii, Wjj, Wij, Wji);
      B.add(i, i, Wii);
      B.add(j, j, Wjj);
      B.add(i, j, Wij);
      B.add(j, i, Wji);
    }
    g->q_cache = std::move(B.out);
    g->q_cache_valid = true;
  }
  const HostBSR& q = g->q_cache;
  *nnzb = static_cast<long long>(q.col.size());
  if (browptr) std::copy(q.rowptr.begin(), q.rowptr.end(), browptr);
  if (bcol) std::copy(q.col.begin(), q.col.end(), bcol);
  if (blocks) std::copy(q.blocks.begin(), q.blocks.end(), blocks);
  return DPGO_HIP_OK;
}

int dpgo_chordal_initialization(int d, int n, int m, const int* p1, const int* p2, const double* R, const double* t,
                                const double* kappa, const double* tau, double* T_out) {
  if ((d != 2 && d != 3) || n <= 0 || m < 0 || !T_out || (m > 0 && (!p1 || !p2 || !R || !t || !kappa || !tau)))
    return fail(DPGO_HIP_EINVAL, "bad chordal initialisation arguments");
  for (int e = 0; e < m; ++e)
    if (p1[e] < 0 || p1[e] >= n || p2[e] < 0 || p2[e] >= n || p1[e] == p2[e])
      return fail(DPGO_HIP_EINVAL, "edge endpoint out of range");
  std::string err;
  if (dpgo::chordal_initialization(d, n, m, p1, p2, R, t, kappa, tau, T_out, err) != 0) return fail(DPGO_HIP_EINVAL, err);
  return DPGO_HIP_OK;
}

int dpgo_graph_chordal_init(dpgo_graph g, int r, const double* YLift, double* X_out) {
  if (!g || !YLift || !X_out) return fail(DPGO_HIP_EINVAL, "null argument");
  const int d = g->d, b = d + 1, n = g->n;
  std::vector<double> T(static_cast<size_t>(n) * d * b);
  DPGO_TRY(dpgo_chordal_initialization(d, n, static_cast<int>(g->p1.size()), g->p1.data(), g->p2.data(), g->R.data(),
                                       g->t.data(), g->kappa.data(), g->tau.data(), T.data()));
  // X = YLift (r x d, column-major) * T (d x b n, column-major)
  for (int p = 0; p < n; ++p)
    for (int c = 0; c < b; ++c)
      for (int a = 0; a < r; ++a) {
        double acc = 0.0;
        for (int u = 0; u < d; ++u) acc += YLift[u * r + a] * T[(static_cast<size_t>(p) * b + c) * d + u];
        X_out[(static_cast<size_t>(p) * b + c) * r + a] = acc;
      }
  return DPGO_HIP_OK;
}

int dpgo_chordal_initialization_gpu(int d, int n, int m, const int* p1, const int* p2, const double* R,
                                    const double* t, const double* kappa, const double* tau, double rtol,
                                    int max_iters, double* T_out, int* iters, double* relres) {
  if ((d != 2 && d != 3) || n <= 0 || m < 0 || !T_out || (m > 0 && (!p1 || !p2 || !R || !t || !kappa || !tau)) ||
      !(rtol > 0.0) || max_iters < 1)
    return fail(DPGO_HIP_EINVAL, "bad chordal initialisation arguments");
  for (int e = 0; e < m; ++e)
    if (p1[e] < 0 || p1[e] >= n || p2[e] < 0 || p2[e] >= n || p1[e] == p2[e])
      return fail(DPGO_HIP_EINVAL, "edge endpoint out of range");
  if (usable_devices() == 0) return fail(DPGO_HIP_ENODEV, "no gfx950 device available (no CPU fallback)");
  std::string err;
  if (dpgo::chordal_initialization_gpu(d, n, m, p1, p2, R, t, kappa, tau, T_out, rtol, max_iters, iters, relres,
                                       err) != 0)
    return fail(DPGO_HIP_EDEVICE, err);
  return DPGO_HIP_OK;
}

int dpgo_graph_chordal_init_gpu(dpgo_graph g, int r, const double* YLift, double rtol, int max_iters,
                                double* X_out, int* iters, double* relres) {
  if (!g || !YLift || !X_out) return fail(DPGO_HIP_EINVAL, "null argument");
  const int d = g->d, b = d + 1, n = g->n;
  std::vector<double> T(static_cast<size_t>(n) * d * b);
  DPGO_TRY(dpgo_chordal_initialization_gpu(d, n, static_cast<int>(g->p1.size()), g->p1.data(), g->p2.data(),
                                           g->R.data(), g->t.data(), g->kappa.data(), g->tau.data(), rtol, max_iters,
                                           T.data(), iters, relres));
  for (int p = 0; p < n; ++p)
    for (int c = 0; c < b; ++c)
      for (int a = 0; a < r; ++a) {
        double acc = 0.0;
        for (int u = 0; u < d; ++u) acc += YLift[u * r + a] * T[(static_cast<size_t>(p) * b + c) * d + u];
        X_out[(static_cast<size_t>(p) * b + c) * r + a] = acc;
      }
  return DPGO_HIP_OK;
}

int dpgo_graph_distributed_init(dpgo_graph g, int num_agents, const int* agent_of_pose, int r, const double* YLift,
                                int use_gpu, double rtol, int max_iters, double* X_out, int* iters, double* relres) {
  if (!g || !YLift || !X_out || !agent_of_pose || num_agents <= 0) return fail(DPGO_HIP_EINVAL, "null argument");
  const int d = g->d, b = d + 1, n = g->n;
  for (int i = 0; i < n; ++i)
    if (agent_of_pose[i] < 0 || agent_of_pose[i] >= num_agents) return fail(DPGO_HIP_EINVAL, "agent_of_pose out of range");
  if (use_gpu && usable_devices() == 0) return fail(DPGO_HIP_ENODEV, "no gfx950 device available (no CPU fallback)");
  if (use_gpu && (!(rtol > 0.0) || max_iters < 1)) return fail(DPGO_HIP_EINVAL, "bad PCG tolerance");
  std::vector<double> T(static_cast<size_t>(n) * d * b);
  std::string err;
  if (dpgo::distributed_initialization(d, n, static_cast<int>(g->p1.size()), g->p1.data(), g->p2.data(), g->R.data(),
                                       g->t.data(), g->kappa.data(), g->tau.data(), agent_of_pose, num_agents,
                                       use_gpu != 0, rtol, max_iters, T.data(), iters, relres, err) != 0)
    return fail(use_gpu ? DPGO_HIP_EDEVICE : DPGO_HIP_EINVAL, err);
  for (int p = 0; p < n; ++p)
    for (int c = 0; c < b; ++c)
      for (int a = 0; a < r; ++a) {
        double acc = 0.0;
        for (int u = 0; u < d; ++u) acc += YLift[u * r + a] * T[(static_cast<size_t>(p) * b + c) * d + u];
        X_out[(static_cast<size_t>(p) * b + c) * r + a] = acc;
      }
  return DPGO_HIP_OK;
}

int dpgo_graph_chain_init(dpgo_graph g, int r, const double* YLift, double* X_out) {
  if (!g || !YLift || !X_out) return fail(DPGO_HIP_EINVAL, "null argument");
  const int d = g->d, b = d + 1, n = g->n;
  // odometry edge for each src (p2 = p1 + 1)
  std::vector<long> odo(n, -1);
  for (size_t e = 0; e < g->p1.size(); ++e)
    if (g->p2[e] == g->p1[e] + 1 && odo[g->p1[e]] < 0) odo[g->p1[e]] = static_cast<long>(e);
  std::vector<double> T(static_cast<size_t>(n) * d * b, 0.0);  // d x b per pose, row-major [u][c]
  for (int u = 0; u < d; ++u) T[u * b + u] = 1.0;
  for (int s = 0; s + 1 < n; ++s) {
    const long e = odo[s];
    const double* Ts = &T[static_cast<size_t>(s) * d * b];
    double* Td = &T[static_cast<size_t>(s + 1) * d * b];
    if (e < 0) {  // chain broken: restart at identity
      for (int u = 0; u < d; ++u) Td[u * b + u] = 1.0;
      continue;
    }
    const double* Rm = &g->R[e * d * d];
    const double* tv = &g->t[e * d];
    for (int u = 0; u < d; ++u) {
      for (int v = 0; v < d; ++v) {
        double acc = 0.0;
        for (int q = 0; q < d; ++q) acc += Ts[u * b + q] * Rm[q * d + v];
        Td[u * b + v] = acc;
      }
      double acc = Ts[u * b + d];
      for (int q = 0; q < d; ++q) acc += Ts[u * b + q] * tv[q];
      Td[u * b + d] = acc;
    }
  }
  // X_j = YLift (r x d, column-major) * T_j (d x b); output pose-major column-major
  for (int j = 0; j < n; ++j)
    for (int c = 0; c < b; ++c)
      for (int a = 0; a < r; ++a) {
        double acc = 0.0;
        for (int u = 0; u < d; ++u) acc += YLift[u * r + a] * T[static_cast<size_t>(j) * d * b + u * b + c];
        X_out[(static_cast<size_t>(j) * b + c) * r + a] = acc;
      }
  return DPGO_HIP_OK;
}

int dpgo_graph_grid_partition(dpgo_graph g, int A, int* agent_of_pose) {
  if (!g || g->coords.empty()) return fail(DPGO_HIP_EINVAL, "not a grid graph");
  int k = 0;
  while (static_cast<long>(k) * k * k < g->n) ++k;
  if (A <= 0 || k % A != 0) return fail(DPGO_HIP_EINVAL, "agents per axis must divide the grid side");
  const int s = k / A;
  for (int i = 0; i < g->n; ++i) {
    const int ax = g->coords[3 * i] / s, ay = g->coords[3 * i + 1] / s, az = g->coords[3 * i + 2] / s;
    agent_of_pose[i] = ax + A * (ay + A * az);
  }
  return DPGO_HIP_OK;
}

}  // extern "C"

// Certified optimality gap of an iterate of the whole graph (the reference has no
// certification, so it is pinned against the oracle's explicit matrices).  X: r x (d+1) n,
// column-major (the reference layout; dpgo_rbcd_get_X's layout).  One single-agent edge-stream handle
// holds the central Q (unit weights); lambda_min(S(X)) by dpgo_hip_certify; f_relax = f(X); the
// rounding follows PGOAgent::getTrajectoryInLocalFrame (src/PGOAgent.cpp:481-498): T = Y_0^T X,
// every rotation block projected to SO(d), translations relative to pose 0; f_rounded = f(T) (T
// lifted by zero rows, which leaves the quadratic form unchanged).  When lambda_min >= -eps the
// relaxation is solved globally and f_relax <= f* <= f_rounded: f_rounded - f_relax bounds the
// rounded trajectory's suboptimality.
int dpgo_graph_certify(dpgo_graph g, int r, const double* X, int max_iters, double tol, double* lambda_min,
                       double* residual, int* iters, double* f_relax, double* f_rounded, double* T_rounded,
                       double* eigvec) {
  dpgo_cert_info info;
  DPGO_TRY(dpgo_graph_certify_ex(g, r, X, max_iters, 0, 0, tol, lambda_min, f_relax, f_rounded, T_rounded, eigvec,
                                 &info));
  if (residual) *residual = info.residual;
  if (iters) *iters = info.iters;
  return DPGO_HIP_OK;
}

int dpgo_graph_certify_ex(dpgo_graph g, int r, const double* X, int max_iters, int basis_max, int flags, double tol,
                          double* lambda_min, double* f_relax, double* f_rounded, double* T_rounded, double* eigvec,
                          dpgo_cert_info* info) {
  if (!g || !X || !lambda_min || r < g->d) return fail(DPGO_HIP_EINVAL, "bad certification arguments");
  const int d = g->d, b = d + 1, n = g->n, m = static_cast<int>(g->p1.size());
  dpgo_hip_problem h = nullptr;
  DPGO_TRY(dpgo_hip_problem_create(n, d, r, &h));
  struct Guard {
    dpgo_hip_problem h;
    ~Guard() { dpgo_hip_problem_destroy(h); }
  } guard{h};
  const std::vector<double> w(static_cast<size_t>(m), 1.0);
  DPGO_TRY(dpgo_hip_set_Q_edges(h, 0, m, g->p1.data(), g->p2.data(), g->R.data(), g->t.data(), g->kappa.data(),
                                g->tau.data(), w.data()));
  DPGO_TRY(dpgo_hip_certify_ex(h, X, max_iters, basis_max, flags, tol, lambda_min, eigvec, info));
  double fx = 0.0;
  DPGO_TRY(dpgo_hip_f(h, X, &fx));
  if (f_relax) *f_relax = fx;
  // rounding: T = Y_0^T X (Y_0 = rows 0..r-1, columns 0..d-1 of X)
  std::vector<double> T(static_cast<size_t>(n) * b * d);
  for (int p = 0; p < n; ++p)
    for (int c = 0; c < b; ++c)
      for (int u = 0; u < d; ++u) {
        double acc = 0.0;
        for (int a = 0; a < r; ++a) acc += X[static_cast<size_t>(u) * r + a] * X[(static_cast<size_t>(p) * b + c) * r + a];
        T[(static_cast<size_t>(p) * b + c) * d + u] = acc;
      }
  double t0[3] = {0.0, 0.0, 0.0};
  for (int u = 0; u < d; ++u) t0[u] = T[static_cast<size_t>(d) * d + u];
  std::vector<double> XT(static_cast<size_t>(n) * b * r, 0.0);
  for (int p = 0; p < n; ++p) {
    double M[9], Rp[9];
    for (int u = 0; u < d; ++u)
      for (int c = 0; c < d; ++c) M[u * d + c] = T[(static_cast<size_t>(p) * b + c) * d + u];
    dpgo::project_to_rotation(d, M, Rp);
    for (int u = 0; u < d; ++u) {
      for (int c = 0; c < d; ++c) T[(static_cast<size_t>(p) * b + c) * d + u] = Rp[u * d + c];
      T[(static_cast<size_t>(p) * b + d) * d + u] -= t0[u];
    }
    for (int c = 0; c < b; ++c)
      for (int u = 0; u < d; ++u) XT[(static_cast<size_t>(p) * b + c) * r + u] = T[(static_cast<size_t>(p) * b + c) * d + u];
  }
  double fr = 0.0;
  DPGO_TRY(dpgo_hip_f(h, XT.data(), &fr));
  if (f_rounded) *f_rounded = fr;
  if (T_rounded) std::memcpy(T_rounded, T.data(), sizeof(double) * T.size());
  return DPGO_HIP_OK;
}

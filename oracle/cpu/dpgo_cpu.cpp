// CPU restatement of one PGOAgent RBCD step -- TEST / BASELINE INFRASTRUCTURE, NOT PRODUCT CODE.
//
// A plain single-threaded C++ restatement (no Eigen / CHOLMOD / ROPTLIB: absent) of
//   PGOAgent::iterate(true) + iterate(false)     src/PGOAgent.cpp:642-718, 1033-1165
//   constructQMatrix / constructGMatrix          src/PGOAgent.cpp:720-859
//   QuadraticProblem f / EucGrad / HVP / precond src/QuadraticProblem.cpp:31-42, 50-101 (block-Jacobi, or the
//                                                exact factor of Q + 0.1 I: RCM + envelope Cholesky)
//   QuadraticOptimizer RTR (1 outer, tCG)        src/QuadraticOptimizer.cpp:34-122 + SURVEY A.4
//   LiftedSEManifold project (one-sided Jacobi)  src/manifold/LiftedSEManifold.cpp:34-45
// Only bench.py's cpu_baseline leg and tests/ use it (via oracle/cpu_port.py): it is the
// timed host-core baseline ("kind": "port") beside the GPU path, never part of the product.
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <map>
#include <set>
#include <vector>

namespace {

// The reference's preconditioner, P = Q + 0.1 I factorised once per Q (src/QuadraticProblem.cpp:31-42, CHOLMOD
// there) and applied as P_X(V P^-1) (:75-87), restated independently of the GPU library's supernodal code: a
// reverse Cuthill-McKee pose order and a dense-row envelope (profile) Cholesky, L's row i stored contiguously from
// its first nonzero column to the diagonal.  Fill stays inside the envelope, so the factor is exact up to rounding.
struct Envelope {
  int N = 0;
  bool ok = false;                 // false: P not positive definite -> the reference's unprojected fallback
  std::vector<int> pose_new;       // old pose -> RCM position
  std::vector<int> first;          // per row: first stored column
  std::vector<size_t> start;       // per row: offset of L(i, first[i])
  std::vector<double> val;
};

struct Agent {
  int d, r, b, n;
  std::vector<int> rowptr, col;      // BSR of Q (block (j,i) column-major)
  std::vector<double> blk, minv;     // blocks, per-pose (Q_jj + 0.1 I)^-1 row-major
  std::vector<int> gpose;            // poses with a G block
  std::vector<double> gblk;          // r*b per entry (column-major)
  std::vector<int> gslot;            // pose -> slot or -1
  bool exact = false;                // precondition with the envelope factor instead of block-Jacobi
  Envelope env;
  size_t L() const { return static_cast<size_t>(n) * r * b; }
};

// Reverse Cuthill-McKee over the pose graph of the BSR pattern: per connected component a BFS from a
// pseudo-peripheral pose (repeated BFS from the last level's minimum-degree pose), neighbours in increasing degree.
std::vector<int> rcm_order(const Agent& A) {
  const int n = A.n;
  std::vector<int> deg(n), order, level(n, -1);
  for (int j = 0; j < n; ++j) deg[j] = A.rowptr[j + 1] - A.rowptr[j];
  std::vector<char> placed(n, 0);
  order.reserve(n);
  auto bfs = [&](int s, std::vector<int>& lv, std::vector<int>& seq) {
    seq.clear();
    lv[s] = 0;
    seq.push_back(s);
    for (size_t h = 0; h < seq.size(); ++h) {
      const int u = seq[h];
      for (int k = A.rowptr[u]; k < A.rowptr[u + 1]; ++k) {
        const int v = A.col[k];
        if (lv[v] < 0 && !placed[v]) {
          lv[v] = lv[u] + 1;
          seq.push_back(v);
        }
      }
    }
  };
  std::vector<int> seq;
  for (int s0 = 0; s0 < n; ++s0) {
    if (placed[s0]) continue;
    int s = s0, ecc = -1;
    for (int pass = 0; pass < 8; ++pass) {  // pseudo-peripheral start
      bfs(s, level, seq);
      const int e = level[seq.back()];
      int best = seq.back();
      for (int v : seq)
        if (level[v] == e && deg[v] < deg[best]) best = v;
      for (int v : seq) level[v] = -1;
      if (e <= ecc) break;
      ecc = e;
      s = best;
    }
    // Cuthill-McKee from s
    const size_t base = order.size();
    order.push_back(s);
    placed[s] = 1;
    for (size_t h = base; h < order.size(); ++h) {
      const int u = order[h];
      std::vector<int> nb;
      for (int k = A.rowptr[u]; k < A.rowptr[u + 1]; ++k)
        if (!placed[A.col[k]]) {
          nb.push_back(A.col[k]);
          placed[A.col[k]] = 1;
        }
      std::stable_sort(nb.begin(), nb.end(), [&](int x, int y) { return deg[x] < deg[y]; });
      order.insert(order.end(), nb.begin(), nb.end());
    }
  }
  std::reverse(order.begin(), order.end());
  std::vector<int> pos(n);
  for (int q = 0; q < n; ++q) pos[order[q]] = q;
  return pos;
}

// P = Q + 0.1 I = L L^T in the envelope of the RCM-ordered pattern (row-oriented, dot products over contiguous rows)
void envelope_factor(Agent& A) {
  Envelope& E = A.env;
  const int b = A.b, bb = b * b, n = A.n;
  E.N = n * b;
  E.pose_new = rcm_order(A);
  E.first.assign(E.N, 0);
  E.start.assign(E.N + 1, 0);
  for (int j = 0; j < n; ++j) {
    int lo = E.pose_new[j];
    for (int k = A.rowptr[j]; k < A.rowptr[j + 1]; ++k) lo = std::min(lo, E.pose_new[A.col[k]]);
    for (int c = 0; c < b; ++c) E.first[E.pose_new[j] * b + c] = lo * b;
  }
  for (int i = 0; i < E.N; ++i) E.start[i + 1] = E.start[i] + static_cast<size_t>(i - E.first[i] + 1);
  E.val.assign(E.start[E.N], 0.0);
  for (int j = 0; j < n; ++j)  // scatter the lower triangle: entry (j b + c, i b + u) = blk[k][u b + c]
    for (int k = A.rowptr[j]; k < A.rowptr[j + 1]; ++k) {
      const int i = A.col[k];
      for (int c = 0; c < b; ++c)
        for (int u = 0; u < b; ++u) {
          const int rn = E.pose_new[j] * b + c, cn = E.pose_new[i] * b + u;
          if (cn <= rn) E.val[E.start[rn] + (cn - E.first[rn])] = A.blk[static_cast<size_t>(k) * bb + u * b + c];
        }
    }
  for (int i = 0; i < E.N; ++i) E.val[E.start[i] + (i - E.first[i])] += 0.1;
  E.ok = true;
  for (int i = 0; i < E.N && E.ok; ++i) {
    double* Li = &E.val[E.start[i]];
    const int fi = E.first[i];
    for (int j = fi; j < i; ++j) {
      const double* Lj = &E.val[E.start[j]];
      const int fj = E.first[j], k0 = std::max(fi, fj);
      double s = Li[j - fi];
      const double* a = Li + (k0 - fi);
      const double* c = Lj + (k0 - fj);
      for (int k = 0; k < j - k0; ++k) s -= a[k] * c[k];
      Li[j - fi] = s / Lj[j - fj];
    }
    double s = Li[i - fi];
    for (int k = 0; k < i - fi; ++k) s -= Li[k] * Li[k];
    if (!(s > 0.0)) {
      E.ok = false;
      break;
    }
    Li[i - fi] = std::sqrt(s);
  }
}

// Z = V P^-1 for the r rows of V at once (pose-major layout), by L y = v, L^T x = y
void envelope_solve(const Agent& A, const double* V, double* Z) {
  const Envelope& E = A.env;
  const int r = A.r, b = A.b, rb = r * b;
  std::vector<double> y(static_cast<size_t>(E.N) * r);
  for (int j = 0; j < A.n; ++j)
    for (int c = 0; c < b; ++c)
      for (int a = 0; a < r; ++a) y[static_cast<size_t>(E.pose_new[j] * b + c) * r + a] = V[static_cast<size_t>(j) * rb + c * r + a];
  for (int i = 0; i < E.N; ++i) {
    const double* Li = &E.val[E.start[i]];
    double acc[8] = {0};
    for (int k = E.first[i]; k < i; ++k) {
      const double l = Li[k - E.first[i]];
      for (int a = 0; a < r; ++a) acc[a] += l * y[static_cast<size_t>(k) * r + a];
    }
    const double inv = 1.0 / Li[i - E.first[i]];
    for (int a = 0; a < r; ++a) y[static_cast<size_t>(i) * r + a] = (y[static_cast<size_t>(i) * r + a] - acc[a]) * inv;
  }
  for (int i = E.N - 1; i >= 0; --i) {
    const double* Li = &E.val[E.start[i]];
    const double inv = 1.0 / Li[i - E.first[i]];
    double x[8];
    for (int a = 0; a < r; ++a) x[a] = y[static_cast<size_t>(i) * r + a] * inv;
    for (int a = 0; a < r; ++a) y[static_cast<size_t>(i) * r + a] = x[a];
    for (int k = E.first[i]; k < i; ++k) {
      const double l = Li[k - E.first[i]];
      for (int a = 0; a < r; ++a) y[static_cast<size_t>(k) * r + a] -= l * x[a];
    }
  }
  for (int j = 0; j < A.n; ++j)
    for (int c = 0; c < b; ++c)
      for (int a = 0; a < r; ++a) Z[static_cast<size_t>(j) * rb + c * r + a] = y[static_cast<size_t>(E.pose_new[j] * b + c) * r + a];
}

inline double dot(const std::vector<double>& a, const std::vector<double>& c) {
  double s = 0.0;
  for (size_t i = 0; i < a.size(); ++i) s += a[i] * c[i];
  return s;
}

void spmm(const Agent& A, const double* X, double* Y) {
  const int r = A.r, b = A.b, rb = r * b;
  for (int j = 0; j < A.n; ++j) {
    double acc[32] = {0};
    for (int k = A.rowptr[j]; k < A.rowptr[j + 1]; ++k) {
      const double* Xi = X + static_cast<size_t>(A.col[k]) * rb;
      const double* B = &A.blk[static_cast<size_t>(k) * b * b];  // block(j,i) col-major = Q_ij row-major
      for (int u = 0; u < b; ++u)       // row u of Q_ij
        for (int c = 0; c < b; ++c) {
          const double q = B[u * b + c];
          for (int a = 0; a < r; ++a) acc[c * r + a] += Xi[u * r + a] * q;
        }
    }
    std::memcpy(Y + static_cast<size_t>(j) * rb, acc, sizeof(double) * rb);
  }
}

// V_Y <- V_Y - Y sym(Y^T V_Y) per pose
void project_pose(int r, int d, const double* X, double* V) {
  double S[9];
  for (int p = 0; p < d; ++p)
    for (int q = 0; q < d; ++q) {
      double s = 0.0;
      for (int a = 0; a < r; ++a) s += X[p * r + a] * V[q * r + a];
      S[p * d + q] = s;
    }
  double Ss[9];
  for (int p = 0; p < d; ++p)
    for (int q = 0; q < d; ++q) Ss[p * d + q] = 0.5 * (S[p * d + q] + S[q * d + p]);
  for (int q = 0; q < d; ++q)
    for (int a = 0; a < r; ++a) {
      double s = V[q * r + a];
      for (int p = 0; p < d; ++p) s -= X[p * r + a] * Ss[p * d + q];
      V[q * r + a] = s;
    }
}

void sym_yt(int r, int d, const double* X, const double* M, double* Ss) {
  double S[9];
  for (int p = 0; p < d; ++p)
    for (int q = 0; q < d; ++q) {
      double s = 0.0;
      for (int a = 0; a < r; ++a) s += X[p * r + a] * M[q * r + a];
      S[p * d + q] = s;
    }
  for (int p = 0; p < d; ++p)
    for (int q = 0; q < d; ++q) Ss[p * d + q] = 0.5 * (S[p * d + q] + S[q * d + p]);
}

void qf_pose(int r, int d, double* M) {  // Gram-Schmidt twice, positive diagonal
  for (int q = 0; q < d; ++q) {
    for (int pass = 0; pass < 2; ++pass)
      for (int p = 0; p < q; ++p) {
        double s = 0.0;
        for (int a = 0; a < r; ++a) s += M[p * r + a] * M[q * r + a];
        for (int a = 0; a < r; ++a) M[q * r + a] -= s * M[p * r + a];
      }
    double nn = 0.0;
    for (int a = 0; a < r; ++a) nn += M[q * r + a] * M[q * r + a];
    const double inv = 1.0 / std::sqrt(nn);
    for (int a = 0; a < r; ++a) M[q * r + a] *= inv;
  }
}

void polar_pose(int r, int d, double* M) {  // one-sided Jacobi SVD -> U V^T
  double V[9] = {0};
  for (int p = 0; p < d; ++p) V[p * d + p] = 1.0;
  for (int sweep = 0; sweep < 30; ++sweep) {
    bool rot = false;
    for (int p = 0; p < d - 1; ++p)
      for (int q = p + 1; q < d; ++q) {
        double al = 0, be = 0, ga = 0;
        for (int a = 0; a < r; ++a) {
          al += M[p * r + a] * M[p * r + a];
          be += M[q * r + a] * M[q * r + a];
          ga += M[p * r + a] * M[q * r + a];
        }
        if (ga != 0.0 && std::fabs(ga) > 1e-17 * std::sqrt(al * be)) {
          rot = true;
          const double z = (be - al) / (2 * ga);
          const double t = std::copysign(1.0, z) / (std::fabs(z) + std::sqrt(1 + z * z));
          const double c = 1 / std::sqrt(1 + t * t), s = c * t;
          for (int a = 0; a < r; ++a) {
            const double mp = M[p * r + a], mq = M[q * r + a];
            M[p * r + a] = c * mp - s * mq;
            M[q * r + a] = s * mp + c * mq;
          }
          for (int a = 0; a < d; ++a) {
            const double vp = V[a * d + p], vq = V[a * d + q];
            V[a * d + p] = c * vp - s * vq;
            V[a * d + q] = s * vp + c * vq;
          }
        }
      }
    if (!rot) break;
  }
  double U[8 * 3];
  for (int q = 0; q < d; ++q) {
    double nn = 0;
    for (int a = 0; a < r; ++a) nn += M[q * r + a] * M[q * r + a];
    const double inv = nn > 0 ? 1 / std::sqrt(nn) : 0;
    for (int a = 0; a < r; ++a) U[q * r + a] = M[q * r + a] * inv;
  }
  for (int q = 0; q < d; ++q)
    for (int a = 0; a < r; ++a) {
      double s = 0;
      for (int p = 0; p < d; ++p) s += U[p * r + a] * V[q * d + p];
      M[q * r + a] = s;
    }
}

struct Work {
  std::vector<double> x1, x2, g, g2, S, S2, eta, Heta, rv, z, delta, Hd, tmp;
  void init(size_t L, size_t SL) {
    for (auto* v : {&x1, &x2, &g, &g2, &eta, &Heta, &rv, &z, &delta, &Hd, &tmp}) v->assign(L, 0.0);
    S.assign(SL, 0.0);
    S2.assign(SL, 0.0);
  }
};

// f, g = P_X(XQ + G), S = sym(Y^T EG_Y); returns f, sets |g|^2
double eval(const Agent& A, const double* X, double* g, double* S, double* ng2, std::vector<double>& tmp) {
  const int r = A.r, d = A.d, b = A.b, rb = r * b;
  spmm(A, X, tmp.data());
  double f = 0.0, gg = 0.0;
  for (int j = 0; j < A.n; ++j) {
    double* EG = &tmp[static_cast<size_t>(j) * rb];
    const double* Xj = X + static_cast<size_t>(j) * rb;
    const int s = A.gslot[j];
    for (int e = 0; e < rb; ++e) {
      const double gv = s >= 0 ? A.gblk[static_cast<size_t>(s) * rb + e] : 0.0;
      f += (0.5 * EG[e] + gv) * Xj[e];
      EG[e] += gv;
    }
    sym_yt(r, d, Xj, EG, S + static_cast<size_t>(j) * d * d);
    double* gj = g + static_cast<size_t>(j) * rb;
    std::memcpy(gj, EG, sizeof(double) * rb);
    const double* Ss = S + static_cast<size_t>(j) * d * d;
    for (int q = 0; q < d; ++q)
      for (int a = 0; a < r; ++a) {
        double v = gj[q * r + a];
        for (int p = 0; p < d; ++p) v -= Xj[p * r + a] * Ss[p * d + q];
        gj[q * r + a] = v;
      }
    for (int e = 0; e < rb; ++e) gg += gj[e] * gj[e];
  }
  *ng2 = gg;
  return f;
}

void hess(const Agent& A, const double* X, const double* S, const double* V, double* H) {
  const int r = A.r, d = A.d, rb = r * A.b;
  spmm(A, V, H);
  for (int j = 0; j < A.n; ++j) {
    double* Hj = H + static_cast<size_t>(j) * rb;
    const double* Vj = V + static_cast<size_t>(j) * rb;
    const double* Ss = S + static_cast<size_t>(j) * d * d;
    for (int q = 0; q < d; ++q)
      for (int a = 0; a < r; ++a) {
        double v = Hj[q * r + a];
        for (int p = 0; p < d; ++p) v -= Vj[p * r + a] * Ss[p * d + q];
        Hj[q * r + a] = v;
      }
    project_pose(r, d, X + static_cast<size_t>(j) * rb, Hj);
  }
}

void precond(const Agent& A, const double* X, const double* V, double* Z) {
  const int r = A.r, d = A.d, b = A.b, rb = r * b;
  if (A.exact) {
    if (!A.env.ok) {  // src/QuadraticProblem.cpp:84-85: factorisation failed -> V itself, unprojected
      std::memcpy(Z, V, sizeof(double) * A.L());
      return;
    }
    envelope_solve(A, V, Z);
    for (int j = 0; j < A.n; ++j) project_pose(r, d, X + static_cast<size_t>(j) * rb, Z + static_cast<size_t>(j) * rb);
    return;
  }
  for (int j = 0; j < A.n; ++j) {
    const double* M = &A.minv[static_cast<size_t>(j) * b * b];
    const double* Vj = V + static_cast<size_t>(j) * rb;
    double* Zj = Z + static_cast<size_t>(j) * rb;
    for (int c = 0; c < b; ++c)
      for (int a = 0; a < r; ++a) {
        double s = 0;
        for (int u = 0; u < b; ++u) s += Vj[u * r + a] * M[u * b + c];
        Zj[c * r + a] = s;
      }
    project_pose(r, d, X + static_cast<size_t>(j) * rb, Zj);
  }
}

// tCG / RTR counters of one optimize call (the layout of dpgo_hip_stats' first ten ints)
struct OptStats {
  int calls = 0, early = 0, runs = 0, tcg_iters = 0, status[5] = {0, 0, 0, 0, 0}, gave_up = 0;
};

// QuadraticOptimizer::optimize with RTR, 1 outer iteration, radius-shrink retries
double optimize(const Agent& A, const double* Xin, double* Xout, int max_inner, double radius, double tol, Work& w,
                OptStats* stats = nullptr) {
  OptStats dummy;
  OptStats& st = stats ? *stats : dummy;
  st.calls += 1;
  const size_t L = A.L();
  const int r = A.r, d = A.d, rb = r * A.b;
  std::memcpy(w.x1.data(), Xin, sizeof(double) * L);
  double ng2;
  const double f1 = eval(A, w.x1.data(), w.g.data(), w.S.data(), &ng2, w.tmp);
  const double ngf = std::sqrt(ng2);
  if (ngf < tol) {
    std::memcpy(Xout, Xin, sizeof(double) * L);
    st.early += 1;
    return f1;
  }
  for (int run = 0; run < 12; ++run) {
    const double Delta = radius;
    std::fill(w.eta.begin(), w.eta.end(), 0.0);
    std::fill(w.Heta.begin(), w.Heta.end(), 0.0);
    w.rv = w.g;
    precond(A, w.x1.data(), w.rv.data(), w.z.data());
    double z_r = dot(w.z, w.rv), d_Pd = z_r, e_Pe = 0, e_Pd = 0;
    const double nr0 = std::sqrt(dot(w.rv, w.rv));
    int status = 4, inner = max_inner;
    for (size_t i = 0; i < L; ++i) w.delta[i] = -w.z[i];
    for (int j = 0; j < max_inner; ++j) {
      hess(A, w.x1.data(), w.S.data(), w.delta.data(), w.Hd.data());
      const double dHd = dot(w.delta, w.Hd);
      const double alpha = z_r / dHd;
      const double ePe_new = e_Pe + 2 * alpha * e_Pd + alpha * alpha * d_Pd;
      if (dHd <= 0 || ePe_new >= Delta * Delta) {
        const double tau = (-e_Pd + std::sqrt(e_Pd * e_Pd + d_Pd * (Delta * Delta - e_Pe))) / d_Pd;
        for (size_t i = 0; i < L; ++i) {
          w.eta[i] += tau * w.delta[i];
          w.Heta[i] += tau * w.Hd[i];
        }
        status = dHd <= 0 ? 0 : 1;
        inner = j + 1;
        break;
      }
      e_Pe = ePe_new;
      for (size_t i = 0; i < L; ++i) {
        w.eta[i] += alpha * w.delta[i];
        w.Heta[i] += alpha * w.Hd[i];
        w.rv[i] += alpha * w.Hd[i];
      }
      const double nr = std::sqrt(dot(w.rv, w.rv));
      if (nr <= nr0 * std::min(nr0, 0.1)) {
        status = 0.1 < nr0 ? 2 : 3;  // LCON / SCON (kappa < |r0|^theta)
        inner = j + 1;
        break;
      }
      precond(A, w.x1.data(), w.rv.data(), w.z.data());
      const double zr_new = dot(w.z, w.rv);
      const double beta = zr_new / z_r;
      for (size_t i = 0; i < L; ++i) w.delta[i] = -w.z[i] + beta * w.delta[i];
      e_Pd = beta * (e_Pd + alpha * d_Pd);
      d_Pd = zr_new + beta * beta * d_Pd;
      z_r = zr_new;
    }
    st.runs += 1;
    st.tcg_iters += inner;
    st.status[status] += 1;
    for (int j = 0; j < A.n; ++j) {
      for (int e = 0; e < rb; ++e) w.x2[j * rb + e] = w.x1[j * rb + e] + w.eta[j * rb + e];
      qf_pose(r, d, &w.x2[static_cast<size_t>(j) * rb]);
    }
    double ng22;
    const double f2 = eval(A, w.x2.data(), w.g2.data(), w.S2.data(), &ng22, w.tmp);
    const double rho = (f1 - f2) / (-dot(w.g, w.eta) - 0.5 * dot(w.eta, w.Heta));
    if (rho > 0.1) {
      std::memcpy(Xout, w.x2.data(), sizeof(double) * L);
      return f2;
    }
    radius /= 4.0;
  }
  st.gave_up += 1;
  std::memcpy(Xout, Xin, sizeof(double) * L);
  return f1;
}

void edge_T(int d, const double* R, const double* t, double T[4][4]) {
  std::memset(T, 0, sizeof(double) * 16);
  for (int u = 0; u < d; ++u) {
    for (int v = 0; v < d; ++v) T[u][v] = R[u * d + v];
    T[u][d] = t[u];
  }
  T[d][d] = 1.0;
}

}  // namespace

extern "C" {

// Times `reps` RBCD steps of one agent (iterate(true) then iterate(false), Nesterov if accel)
// on one host thread.  X is the global r x (d+1) n matrix in column-major layout.
// Returns seconds per agent step; f_out receives f after the last optimisation.
double dpgo_cpu_time_agent_step(int d, int r, int m, const int* p1, const int* p2, const double* R, const double* t,
                                const double* kappa, const double* tau, int n, const int* agent_of_pose, int agent,
                                const double* Xg, int accel, int num_agents, int reps, double* f_out) {
  const int b = d + 1, rb = r * b;
  Agent A;
  A.d = d;
  A.r = r;
  A.b = b;
  std::vector<int> local(n, -1), poses;
  for (int i = 0; i < n; ++i)
    if (agent_of_pose[i] == agent) {
      local[i] = static_cast<int>(poses.size());
      poses.push_back(i);
    }
  A.n = static_cast<int>(poses.size());
  // ---- Q (constructQMatrix) as a map of blocks
  std::vector<std::map<int, std::vector<double>>> rows(A.n);
  auto add = [&](int i, int j, const double* blkcm) {
    auto& v = rows[i][j];
    if (v.empty()) v.assign(b * b, 0.0);
    for (int q = 0; q < b * b; ++q) v[q] += blkcm[q];
  };
  std::map<int, std::vector<double>> G;
  for (int e = 0; e < m; ++e) {
    const int i = p1[e], j = p2[e];
    const bool oi = agent_of_pose[i] == agent, oj = agent_of_pose[j] == agent;
    if (!oi && !oj) continue;
    double T[4][4], Om[4];
    edge_T(d, &R[e * d * d], &t[e * d], T);
    for (int u = 0; u < d; ++u) Om[u] = kappa[e];
    Om[d] = tau[e];
    double Wii[16], Wjj[16], Wij[16], Wji[16];
    for (int u = 0; u < b; ++u)
      for (int v = 0; v < b; ++v) {
        double s = 0;
        for (int q = 0; q < b; ++q) s += T[u][q] * Om[q] * T[v][q];
        Wii[v * b + u] = s;
        Wjj[v * b + u] = u == v ? Om[u] : 0.0;
        Wij[v * b + u] = -T[u][v] * Om[v];
        Wji[v * b + u] = -Om[u] * T[v][u];
      }
    if (oi && oj) {
      add(local[i], local[i], Wii);
      add(local[j], local[j], Wjj);
      add(local[i], local[j], Wij);
      add(local[j], local[i], Wji);
    } else {
      // constructGMatrix (:783-859) from the neighbour's current pose
      const int own = oi ? i : j, nbr = oi ? j : i;
      if (oi)
        add(local[i], local[i], Wii);
      else
        add(local[j], local[j], Wjj);
      auto& gv = G[local[own]];
      if (gv.empty()) gv.assign(rb, 0.0);
      const double* Xn = Xg + static_cast<size_t>(nbr) * rb;
      // L = -X_n Om T^T (outgoing) or -X_n T Om (incoming); X_n is r x b column-major
      for (int c = 0; c < b; ++c)
        for (int a = 0; a < r; ++a) {
          double s = 0;
          for (int u = 0; u < b; ++u) s += Xn[u * r + a] * (oi ? Om[u] * T[c][u] : T[u][c] * Om[c]);
          gv[c * r + a] -= s;
        }
    }
  }
  A.rowptr.assign(A.n + 1, 0);
  for (int j = 0; j < A.n; ++j) {
    if (rows[j].find(j) == rows[j].end()) rows[j][j].assign(b * b, 0.0);
    A.rowptr[j + 1] = A.rowptr[j] + static_cast<int>(rows[j].size());
    for (auto& kv : rows[j]) {
      A.col.push_back(kv.first);
      A.blk.insert(A.blk.end(), kv.second.begin(), kv.second.end());
    }
  }
  // block-Jacobi inverses (Gauss-Jordan)
  A.minv.assign(static_cast<size_t>(A.n) * b * b, 0.0);
  for (int j = 0; j < A.n; ++j) {
    double M[4][8] = {{0}};
    const double* D = rows[j][j].data();
    for (int u = 0; u < b; ++u) {
      for (int v = 0; v < b; ++v) M[u][v] = D[v * b + u];
      M[u][u] += 0.1;
      M[u][b + u] = 1.0;
    }
    for (int c = 0; c < b; ++c) {
      int piv = c;
      for (int u = c + 1; u < b; ++u)
        if (std::fabs(M[u][c]) > std::fabs(M[piv][c])) piv = u;
      for (int v = 0; v < 2 * b; ++v) std::swap(M[c][v], M[piv][v]);
      const double inv = 1.0 / M[c][c];
      for (int v = 0; v < 2 * b; ++v) M[c][v] *= inv;
      for (int u = 0; u < b; ++u)
        if (u != c) {
          const double f = M[u][c];
          for (int v = 0; v < 2 * b; ++v) M[u][v] -= f * M[c][v];
        }
    }
    for (int u = 0; u < b; ++u)
      for (int v = 0; v < b; ++v) A.minv[static_cast<size_t>(j) * b * b + u * b + v] = M[u][b + v];
  }
  A.gslot.assign(A.n, -1);
  for (auto& kv : G) {
    A.gslot[kv.first] = static_cast<int>(A.gpose.size());
    A.gpose.push_back(kv.first);
    A.gblk.insert(A.gblk.end(), kv.second.begin(), kv.second.end());
  }
  // ---- agent state
  const size_t L = A.L();
  std::vector<double> X(L), Y(L), V(L), Xp(L), M(L);
  for (int q = 0; q < A.n; ++q) std::memcpy(&X[static_cast<size_t>(q) * rb], Xg + static_cast<size_t>(poses[q]) * rb, sizeof(double) * rb);
  Y = X;
  V = X;
  Work w;
  w.init(L, static_cast<size_t>(A.n) * d * d);
  double gamma = 0, alpha = 0, f = 0;
  const double N = num_agents;
  auto t0 = std::chrono::steady_clock::now();
  for (int rep = 0; rep < reps; ++rep) {
    for (int sel = 1; sel >= 0; --sel) {  // iterate(true), then iterate(false)
      Xp = X;
      if (accel) {
        gamma = (1 + std::sqrt(1 + 4 * N * N * gamma * gamma)) / (2 * N);
        alpha = 1 / (gamma * N);
        for (size_t i = 0; i < L; ++i) Y[i] = (1 - alpha) * X[i] + alpha * V[i];
        for (int j = 0; j < A.n; ++j) polar_pose(r, d, &Y[static_cast<size_t>(j) * rb]);
        if (sel)
          f = optimize(A, Y.data(), X.data(), 10, 100.0, 1e-2, w);
        else
          X = Y;
        for (size_t i = 0; i < L; ++i) V[i] = V[i] + gamma * (X[i] - Y[i]);
        for (int j = 0; j < A.n; ++j) polar_pose(r, d, &V[static_cast<size_t>(j) * rb]);
      } else if (sel) {
        f = optimize(A, X.data(), X.data(), 10, 100.0, 1e-2, w);
      }
    }
  }
  const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (f_out) *f_out = f;
  return sec / reps;
}

}  // extern "C"

// =============================================================================================
// Multi-agent colour-schedule RBCD on the host: the CPU restatement of the engine's schedule
// (oracle.colour_rbcd, PGOAgent::iterate src/PGOAgent.cpp:642-718 for every agent, L2 cost,
// block-Jacobi), single-threaded or OpenMP over the agents of a colour class.  Baseline and
// full-scale parity infrastructure only.
// =============================================================================================
namespace {

struct SharedEdge {
  int own;        // agent-local pose
  long nbr;       // global neighbour pose
  int outgoing;   // the agent owns p1
  double T[4][4], Om[4];
};

struct CpuAgent {
  Agent A;
  std::vector<long> poses;  // global ids, local order
  std::vector<int> edges;   // global edge ids touching the agent (private and shared)
  std::vector<double> w;    // this agent's weight per entry of edges (its own copy of a shared edge's)
  // neighborPoseDict (src/PGOAgent.cpp:1201-1235): per entry of `edges` that is a shared loop closure, the neighbour's
  // pose as this agent last received it (snapshot when the agent is selected, examples/MultiRobotExample.cpp:188-213),
  // and whether it ever did; a reweighting reads only these
  std::vector<double> dict;
  std::vector<char> have;
  std::vector<SharedEdge> shared;
  OptStats st;
  double status_rel = 0.0;
  double conv_ratio = 1.0;  // computeConvergedLoopClosureRatio (GNC_TLS)
  int ready = 0;
  bool factored = false;    // exact preconditioner: P = Q + 0.1 I factorised for the current Q
  double factor_sec = 0.0;  // wall seconds of this agent's factorisations
  int factor_count = 0;
};

struct CpuEngine {
  int d = 0, r = 0, b = 0, K = 0, C = 0, accel = 0, restart = 30;
  long n = 0;
  std::vector<int> color;
  std::vector<CpuAgent> ag;
  std::vector<double> X, Y, V, XP;  // global, r b doubles per pose
  double gamma = 0.0, alpha = 0.0;
  long iteration = 0;
  std::vector<Work> work;  // per thread
  // the graph (kept for the robust cost's reweighting and Q rebuilds)
  int m = 0;
  std::vector<int> p1, p2, agent_of, local;
  std::vector<double> R, t, kappa, tau;
  // robust cost (0: L2, 1: GNC_TLS; RobustCostParameters / PGOAgentParameters defaults)
  int robust = 0, inner_iters = 30, gnc_max_iters = 100, gnc_iter = 0;
  int precon_exact = 0;  // the reference's preconditioner (envelope factor of Q + 0.1 I) instead of block-Jacobi
  double mu = 1e-4, mu_step = 1.4, barc = 10.0, min_ratio = 0.8;
  size_t rb() const { return static_cast<size_t>(r) * b; }
};

// Q (private edges + shared-edge diagonal terms), block-Jacobi inverses, shared edges and G slots of agent
// a from its edge list, with weights w (per entry of `edges`; nullptr = 1): PGOAgent::constructQMatrix
void build_agent(int d, int r, int m, const int* p1, const int* p2, const double* R, const double* t, const double* kappa,
                 const double* tau, const int* agent_of, const std::vector<int>& local, int a,
                 const std::vector<int>& edges, CpuAgent& out, const double* w = nullptr) {
  const int b = d + 1, bb = b * b, rb = r * b;
  (void)m;
  Agent& A = out.A;
  out.shared.clear();
  A.gpose.clear();
  A.d = d;
  A.r = r;
  A.b = b;
  A.n = static_cast<int>(out.poses.size());
  struct Trip {
    int i, j;
    double blk[16];
  };
  std::vector<Trip> trips;
  trips.reserve(edges.size() * 3 + A.n);
  for (int j = 0; j < A.n; ++j) {
    Trip tz{j, j, {0}};
    trips.push_back(tz);
  }
  for (size_t q = 0; q < edges.size(); ++q) {
    const int e = edges[q];
    const int i = p1[e], j = p2[e];
    const bool oi = agent_of[i] == a, oj = agent_of[j] == a;
    const double we = w ? w[q] : 1.0;
    double T[4][4], Om[4];
    edge_T(d, &R[static_cast<size_t>(e) * d * d], &t[static_cast<size_t>(e) * d], T);
    for (int u = 0; u < d; ++u) Om[u] = we * kappa[e];
    Om[d] = we * tau[e];
    Trip ii{local[i], local[i], {0}}, jj{local[j], local[j], {0}}, ij{local[i], local[j], {0}}, ji{local[j], local[i], {0}};
    for (int u = 0; u < b; ++u)
      for (int v = 0; v < b; ++v) {
        double s = 0;
        for (int q = 0; q < b; ++q) s += T[u][q] * Om[q] * T[v][q];
        ii.blk[v * b + u] = s;  // column-major blocks (block (j, i) col-major = Q_ij row-major)
        jj.blk[v * b + u] = u == v ? Om[u] : 0.0;
        ij.blk[v * b + u] = -T[u][v] * Om[v];
        ji.blk[v * b + u] = -Om[u] * T[v][u];
      }
    if (oi && oj) {
      trips.push_back(ii);
      trips.push_back(jj);
      trips.push_back(ij);
      trips.push_back(ji);
    } else {
      SharedEdge se;
      se.outgoing = oi ? 1 : 0;
      se.own = oi ? local[i] : local[j];
      se.nbr = oi ? j : i;
      std::memcpy(se.T, T, sizeof(T));
      std::memcpy(se.Om, Om, sizeof(Om));
      out.shared.push_back(se);
      trips.push_back(oi ? ii : jj);
    }
  }
  std::stable_sort(trips.begin(), trips.end(), [](const Trip& x, const Trip& y) { return x.i != y.i ? x.i < y.i : x.j < y.j; });
  A.rowptr.assign(A.n + 1, 0);
  A.col.clear();
  A.blk.clear();
  for (size_t k = 0; k < trips.size(); ++k) {
    const Trip& tr = trips[k];
    if (k > 0 && trips[k - 1].i == tr.i && trips[k - 1].j == tr.j) {  // same block: accumulate
      double* dst = &A.blk[A.blk.size() - bb];
      for (int x = 0; x < bb; ++x) dst[x] += tr.blk[x];
    } else {
      A.col.push_back(tr.j);
      A.blk.insert(A.blk.end(), tr.blk, tr.blk + bb);
    }
    A.rowptr[tr.i + 1] = static_cast<int>(A.col.size());
  }
  // block-Jacobi inverses (Gauss-Jordan) of the diagonal blocks + 0.1 I
  A.minv.assign(static_cast<size_t>(A.n) * bb, 0.0);
  for (int j = 0; j < A.n; ++j) {
    double M[4][8] = {{0}};
    for (int k = A.rowptr[j]; k < A.rowptr[j + 1]; ++k)
      if (A.col[k] == j)
        for (int u = 0; u < b; ++u)
          for (int v = 0; v < b; ++v) M[u][v] = A.blk[static_cast<size_t>(k) * bb + v * b + u];
    for (int u = 0; u < b; ++u) {
      M[u][u] += 0.1;
      M[u][b + u] = 1.0;
    }
    for (int c = 0; c < b; ++c) {
      int piv = c;
      for (int u = c + 1; u < b; ++u)
        if (std::fabs(M[u][c]) > std::fabs(M[piv][c])) piv = u;
      for (int v = 0; v < 2 * b; ++v) std::swap(M[c][v], M[piv][v]);
      const double inv = 1.0 / M[c][c];
      for (int v = 0; v < 2 * b; ++v) M[c][v] *= inv;
      for (int u = 0; u < b; ++u)
        if (u != c) {
          const double f = M[u][c];
          for (int v = 0; v < 2 * b; ++v) M[u][v] -= f * M[c][v];
        }
    }
    for (int u = 0; u < b; ++u)
      for (int v = 0; v < b; ++v) A.minv[static_cast<size_t>(j) * bb + u * b + v] = M[u][b + v];
  }
  // G slots: the public poses (fixed structure)
  A.gslot.assign(A.n, -1);
  for (const auto& se : out.shared)
    if (A.gslot[se.own] < 0) {
      A.gslot[se.own] = static_cast<int>(A.gpose.size());
      A.gpose.push_back(se.own);
    }
  A.gblk.assign(A.gpose.size() * rb, 0.0);
}

// constructGMatrix (:783-859) from the neighbours' current global poses
void assemble_G(CpuAgent& c, const std::vector<double>& Xg, int r, int b) {
  const int rb = r * b;
  std::fill(c.A.gblk.begin(), c.A.gblk.end(), 0.0);
  for (const auto& se : c.shared) {
    double* gv = &c.A.gblk[static_cast<size_t>(c.A.gslot[se.own]) * rb];
    const double* Xn = &Xg[static_cast<size_t>(se.nbr) * rb];
    for (int cc = 0; cc < b; ++cc)
      for (int a = 0; a < r; ++a) {
        double s = 0;
        for (int u = 0; u < b; ++u) s += Xn[u * r + a] * (se.outgoing ? se.Om[u] * se.T[cc][u] : se.T[u][cc] * se.Om[cc]);
        gv[cc * r + a] -= s;
      }
  }
}

void gather(const CpuAgent& c, const std::vector<double>& G, std::vector<double>& out, size_t rb) {
  out.resize(c.poses.size() * rb);
  for (size_t q = 0; q < c.poses.size(); ++q)
    std::memcpy(&out[q * rb], &G[static_cast<size_t>(c.poses[q]) * rb], sizeof(double) * rb);
}

void scatter(const CpuAgent& c, const std::vector<double>& in, std::vector<double>& G, size_t rb) {
  for (size_t q = 0; q < c.poses.size(); ++q)
    std::memcpy(&G[static_cast<size_t>(c.poses[q]) * rb], &in[q * rb], sizeof(double) * rb);
}

void project_all(std::vector<double>& M, int r, int d, size_t rb) {
  for (size_t q = 0; q < M.size() / rb; ++q) polar_pose(r, d, &M[q * rb]);
}

// RobustCost::weight for GNC_TLS (src/DPGO_robust.cpp:23-67) at the engine's mu
double gnc_tls_weight(const CpuEngine& E, double rr) {
  const double rsq = rr * rr, bc = E.barc * E.barc, mu = E.mu;
  if (rsq >= (mu + 1) / mu * bc) return 0.0;
  if (rsq <= mu / (mu + 1) * bc) return 1.0;
  return std::sqrt(bc * mu * (mu + 1) / rsq) - mu;
}

// computeMeasurementError (src/DPGO_utils.cpp:509-515) of edge e between the poses Xi (p1) and Xj (p2)
double measurement_error(const CpuEngine& E, int e, const double* Xi, const double* Xj) {
  const int d = E.d, r = E.r;
  const double* Rm = &E.R[static_cast<size_t>(e) * d * d];
  const double* tv = &E.t[static_cast<size_t>(e) * d];
  double rot = 0.0, tr = 0.0;
  for (int a = 0; a < r; ++a) {
    for (int c = 0; c < d; ++c) {  // (Y1 R - Y2)[a][c]; Y column c = X[c * r + a]
      double s = -Xj[c * r + a];
      for (int u = 0; u < d; ++u) s += Xi[u * r + a] * Rm[u * d + c];
      rot += s * s;
    }
    double s = Xj[d * r + a] - Xi[d * r + a];  // p2 - p1 - Y1 t
    for (int u = 0; u < d; ++u) s -= Xi[u * r + a] * tv[u];
    tr += s * s;
  }
  return E.kappa[e] * rot + E.tau[e] * tr;
}

// neighborPoseDict update of a selected agent (examples/MultiRobotExample.cpp:188-213: the driver hands the selected
// robot its neighbours' public poses): every shared edge's other endpoint, as the neighbours hold it now
void snapshot_neighbors(CpuEngine& E, int a) {
  CpuAgent& c = E.ag[a];
  const size_t rb = E.rb();
  for (size_t q = 0; q < c.edges.size(); ++q) {
    const int e = c.edges[q], i = E.p1[e], j = E.p2[e];
    if (E.agent_of[i] == E.agent_of[j]) continue;
    const long nb = E.agent_of[i] == a ? j : i;
    std::memcpy(&c.dict[q * rb], &E.X[static_cast<size_t>(nb) * rb], sizeof(double) * rb);
    c.have[q] = 1;
  }
}

// PGOAgent::updateLoopClosuresWeights (src/PGOAgent.cpp:1181-1244) then constructQMatrix: private loop
// closures (not odometry: consecutive local indices) at the agent's own X, and the shared ones this agent owns the
// update of (the other agent has the larger ID) against the neighbour's pose in the agent's own
// dictionary -- an edge whose neighbour pose it never received keeps its weight ("cannot update edge"); plus the
// converged ratio.
void reweight_agent(CpuEngine& E, int a) {
  CpuAgent& c = E.ag[a];
  const size_t rb = E.rb();
  long lc = 0, conv = 0;
  for (size_t q = 0; q < c.edges.size(); ++q) {
    const int e = c.edges[q], i = E.p1[e], j = E.p2[e];
    const int ai = E.agent_of[i], aj = E.agent_of[j];
    const double* Xi = &E.X[static_cast<size_t>(i) * rb];
    const double* Xj = &E.X[static_cast<size_t>(j) * rb];
    if (ai == aj) {
      if (E.local[j] == E.local[i] + 1) continue;  // odometry: never reweighted, not a loop closure
    } else if ((ai == a ? aj : ai) < a) {
      ++lc;  // the other agent updates it; this copy keeps its weight
      conv += (c.w[q] == 1.0 || c.w[q] == 0.0) ? 1 : 0;
      continue;
    } else {
      if (!c.have[q]) {  // not in neighborPoseDict: "cannot update edge", the weight stays
        ++lc;
        conv += (c.w[q] == 1.0 || c.w[q] == 0.0) ? 1 : 0;
        continue;
      }
      (ai == a ? Xj : Xi) = &c.dict[q * rb];
    }
    c.w[q] = gnc_tls_weight(E, std::sqrt(measurement_error(E, e, Xi, Xj)));
    ++lc;
    conv += (c.w[q] == 1.0 || c.w[q] == 0.0) ? 1 : 0;
  }
  c.conv_ratio = lc ? static_cast<double>(conv) / static_cast<double>(lc) : std::nan("");
  build_agent(E.d, E.r, E.m, E.p1.data(), E.p2.data(), E.R.data(), E.t.data(), E.kappa.data(), E.tau.data(),
              E.agent_of.data(), E.local, a, c.edges, c, c.w.data());
  c.A.exact = E.precon_exact != 0;  // setQ refactorises P = Q + 0.1 I (src/QuadraticProblem.cpp:31-42): at the
  c.factored = false;                // agent's next optimize (ensure_factor), the only place the factor is read
}

// The factor of the agent's current Q, computed when an optimize call first needs it (timed per agent)
void ensure_factor(CpuAgent& c) {
  if (!c.A.exact || c.factored) return;
  const auto t0 = std::chrono::steady_clock::now();
  envelope_factor(c.A);
  c.factor_sec += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  c.factor_count += 1;
  c.factored = true;
}

// PGOAgent::iterate for agent a (selected or not) on the global state; gamma / alpha already updated
void iterate_agent(CpuEngine& E, int a, bool selected, bool restart, Work& w, bool reweight = false) {
  CpuAgent& c = E.ag[a];
  const size_t rb = E.rb();
  if (selected && E.robust) snapshot_neighbors(E, a);  // this iteration's neighbour poses, before any reweighting
  if (reweight) {  // shouldUpdateLoopClosureWeights: reweight, then initializeAcceleration (XPrev = V = Y = X)
    reweight_agent(E, a);
    if (E.accel)
      for (long p : c.poses) {
        std::memcpy(&E.V[static_cast<size_t>(p) * rb], &E.X[static_cast<size_t>(p) * rb], sizeof(double) * rb);
        std::memcpy(&E.Y[static_cast<size_t>(p) * rb], &E.X[static_cast<size_t>(p) * rb], sizeof(double) * rb);
      }
  }
  if (selected && w.x1.size() != c.A.L()) w.init(c.A.L(), static_cast<size_t>(c.A.n) * E.d * E.d);
  if (selected) ensure_factor(c);
  std::vector<double> X, Y, V, XP;
  gather(c, E.X, X, rb);
  XP = X;  // XPrev = X (:673)
  if (E.accel) {
    gather(c, E.V, V, rb);
    Y.resize(X.size());
    for (size_t i = 0; i < X.size(); ++i) Y[i] = (1.0 - E.alpha) * X[i] + E.alpha * V[i];  // updateY
    project_all(Y, E.r, E.d, rb);
    if (selected) {
      assemble_G(c, E.X, E.r, E.b);  // neighbours' aux poses = their X after iterate(false)
      optimize(c.A, Y.data(), X.data(), 10, 100.0, 1e-2, w, &c.st);
    } else {
      X = Y;  // updateX(false, true)
    }
    for (size_t i = 0; i < X.size(); ++i) V[i] = V[i] + E.gamma * (X[i] - Y[i]);  // updateV
    project_all(V, E.r, E.d, rb);
    if (restart) {  // restartNesterovAcceleration (:1040-1060)
      X = XP;
      if (selected) {
        assemble_G(c, E.X, E.r, E.b);
        optimize(c.A, X.data(), X.data(), 10, 100.0, 1e-2, w, &c.st);
      }
      V = X;
      Y = X;
    }
    scatter(c, V, E.V, rb);
    scatter(c, Y, E.Y, rb);
  } else if (selected) {
    assemble_G(c, E.X, E.r, E.b);
    optimize(c.A, X.data(), X.data(), 10, 100.0, 1e-2, w, &c.st);
  }
  if (selected) {  // status (:700-716)
    double s = 0.0;
    for (size_t i = 0; i < X.size(); ++i) s += (X[i] - XP[i]) * (X[i] - XP[i]);
    c.status_rel = std::sqrt(s / static_cast<double>(c.poses.size()));
    c.ready = (c.status_rel > 5e-3 || (E.robust && c.conv_ratio < E.min_ratio)) ? 0 : 1;
  }
  scatter(c, X, E.X, rb);
}

}  // namespace

extern "C" {

// robust: 0 = L2, 1 = GNC_TLS (reweighting every robust_inner_iters iterations, mu from 1e-4 by 1.4 per
// reweighting for at most 100, barc 10, converged-ratio threshold 0.8: the PGOAgentParameters defaults)
// precon_exact: 1 = the reference's preconditioner (factor of Q + 0.1 I, refactorised whenever Q changes), 0 =
// block-Jacobi
void* dpgo_cpu_rbcd_create(int d, int r, int m, const int* p1, const int* p2, const double* R, const double* t,
                           const double* kappa, const double* tau, long n, const int* agent_of_pose, int num_agents,
                           int accel, int restart_interval, int robust, int robust_inner_iters, int precon_exact) {
  auto* E = new CpuEngine();
  E->precon_exact = precon_exact;
  E->robust = robust;
  E->inner_iters = robust_inner_iters > 0 ? robust_inner_iters : 30;
  E->m = m;
  E->p1.assign(p1, p1 + m);
  E->p2.assign(p2, p2 + m);
  E->R.assign(R, R + static_cast<size_t>(m) * d * d);
  E->t.assign(t, t + static_cast<size_t>(m) * d);
  E->kappa.assign(kappa, kappa + m);
  E->tau.assign(tau, tau + m);
  E->agent_of.assign(agent_of_pose, agent_of_pose + n);
  E->d = d;
  E->r = r;
  E->b = d + 1;
  E->n = n;
  E->K = num_agents;
  E->accel = accel;
  E->restart = restart_interval;
  std::vector<int> local(n);
  E->ag.resize(num_agents);
  for (long i = 0; i < n; ++i) {
    const int a = agent_of_pose[i];
    local[i] = static_cast<int>(E->ag[a].poses.size());
    E->ag[a].poses.push_back(i);
  }
  std::vector<std::vector<int>> edges(num_agents);
  std::vector<std::set<int>> adj(num_agents);
  for (int e = 0; e < m; ++e) {
    const int a1 = agent_of_pose[p1[e]], a2 = agent_of_pose[p2[e]];
    edges[a1].push_back(e);
    if (a2 != a1) {
      edges[a2].push_back(e);
      adj[a1].insert(a2);
      adj[a2].insert(a1);
    }
  }
  // greedy colouring in agent-id order (the engine's and oracle.greedy_colors')
  E->color.assign(num_agents, -1);
  for (int a = 0; a < num_agents; ++a) {
    std::set<int> used;
    for (int nb : adj[a])
      if (E->color[nb] >= 0) used.insert(E->color[nb]);
    int c = 0;
    while (used.count(c)) ++c;
    E->color[a] = c;
    E->C = std::max(E->C, c + 1);
  }
  E->local = local;
#pragma omp parallel for schedule(dynamic)
  for (int a = 0; a < num_agents; ++a) {
    E->ag[a].edges = edges[a];
    E->ag[a].w.assign(edges[a].size(), 1.0);
    E->ag[a].dict.assign(robust ? edges[a].size() * static_cast<size_t>(r) * (d + 1) : 0, 0.0);
    E->ag[a].have.assign(edges[a].size(), 0);
    build_agent(d, r, m, p1, p2, R, t, kappa, tau, agent_of_pose, local, a, edges[a], E->ag[a]);
    E->ag[a].A.exact = precon_exact != 0;
  }
  const size_t L = static_cast<size_t>(n) * E->rb();
  E->X.assign(L, 0.0);
  E->Y.assign(L, 0.0);
  E->V.assign(L, 0.0);
  // one workspace per thread of the widest team an iterate may request (a colour's agents: the all-cores leg)
  E->work.resize(std::max(32, omp_get_max_threads()));
  return E;
}

void dpgo_cpu_rbcd_destroy(void* h) { delete static_cast<CpuEngine*>(h); }

// PGOAgent::setX for every agent: X, and Nesterov restarted (V = Y = X, gamma = alpha = 0)
void dpgo_cpu_rbcd_set_X(void* h, const double* Xg) {
  auto* E = static_cast<CpuEngine*>(h);
  std::memcpy(E->X.data(), Xg, sizeof(double) * E->X.size());
  E->Y = E->X;
  E->V = E->X;
  E->gamma = E->alpha = 0.0;
  E->iteration = 0;
}

// Rounding-noise model for parity bars (test infrastructure): every entry of X, Y and V multiplied by (1 + eps u),
// u uniform in [-1, 1) from SplitMix64(seed), WITHOUT touching the Nesterov state (set_X would restart it).  Applied
// after every iteration at eps ~ 1e-16 it stands for an implementation whose rounding differs from this one's in
// every step -- the GPU's -- so "port vs port-with-noise" measures how far the trajectory itself carries such
// differences.
void dpgo_cpu_rbcd_perturb(void* h, double eps, unsigned long long seed) {
  auto* E = static_cast<CpuEngine*>(h);
  unsigned long long z = seed;
  auto next = [&z]() {
    unsigned long long x = (z += 0x9E3779B97F4A7C15ULL);
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
  };
  for (auto* v : {&E->X, &E->Y, &E->V})
    for (double& x : *v) x *= 1.0 + eps * (static_cast<double>(next() >> 11) * 0x1.0p-52 - 1.0);
}

void dpgo_cpu_rbcd_get_X(void* h, double* Xg) {
  auto* E = static_cast<CpuEngine*>(h);
  std::memcpy(Xg, E->X.data(), sizeof(double) * E->X.size());
}

// One colour iteration (colour = iteration mod C) with `threads` OpenMP threads over each phase's
// agents.  upd_sec (optional, [num_agents]): wall seconds of each selected agent's iterate(true).
// timed_serial > 0: the first timed_serial selected agents run one after another on one thread
// (each timed alone), the rest in parallel.  Returns the iteration's wall seconds.
double dpgo_cpu_rbcd_iterate(void* h, int threads, double* upd_sec, int timed_serial) {
  auto* E = static_cast<CpuEngine*>(h);
  const auto t0 = std::chrono::steady_clock::now();
  const int c = static_cast<int>(E->iteration % E->C);
  E->iteration += 1;
  const bool restart = E->accel && ((E->iteration + 1) % E->restart == 0);
  // shouldUpdateLoopClosureWeights (:1174-1179): every agent reweights at the start of its iterate (the
  // non-selected ones first, the selected ones after them, on the poses their neighbours then hold), all
  // with this mu; RobustCost::update once afterwards; with acceleration each restarts Nesterov
  const bool gnc = E->robust && (E->iteration + 1) % E->inner_iters == 0;
  if (gnc && E->accel) E->gamma = E->alpha = 0.0;
  if (E->accel) {
    const double N = E->K;
    E->gamma = (1 + std::sqrt(1 + 4 * N * N * E->gamma * E->gamma)) / (2 * N);
    E->alpha = 1 / (E->gamma * N);
  }
  std::vector<int> sel, oth;
  for (int a = 0; a < E->K; ++a) (E->color[a] == c ? sel : oth).push_back(a);
  const int T = std::max(1, std::min(threads, static_cast<int>(E->work.size())));
#pragma omp parallel for num_threads(T) schedule(dynamic)
  for (int q = 0; q < static_cast<int>(oth.size()); ++q)
    iterate_agent(*E, oth[q], false, restart, E->work[omp_get_thread_num()], gnc);
  const int ns = std::min<int>(std::max(timed_serial, 0), static_cast<int>(sel.size()));
  for (int q = 0; q < ns; ++q) {
    const auto u0 = std::chrono::steady_clock::now();
    iterate_agent(*E, sel[q], true, restart, E->work[0], gnc);
    if (upd_sec) upd_sec[sel[q]] = std::chrono::duration<double>(std::chrono::steady_clock::now() - u0).count();
  }
#pragma omp parallel for num_threads(T) schedule(dynamic)
  for (int q = ns; q < static_cast<int>(sel.size()); ++q) {
    const auto u0 = std::chrono::steady_clock::now();
    iterate_agent(*E, sel[q], true, restart, E->work[omp_get_thread_num()], gnc);
    if (upd_sec) upd_sec[sel[q]] = std::chrono::duration<double>(std::chrono::steady_clock::now() - u0).count();
  }
  if (gnc && ++E->gnc_iter <= E->gnc_max_iters) E->mu *= E->mu_step;  // RobustCost::update (:86-103)
  if (restart) E->gamma = E->alpha = 0.0;
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// per agent: calls, early, runs, tcg_iters, status[5], gave_up (dpgo_hip_stats' first ten)
void dpgo_cpu_rbcd_stats(void* h, int* out) {
  auto* E = static_cast<CpuEngine*>(h);
  for (int a = 0; a < E->K; ++a) {
    const OptStats& s = E->ag[a].st;
    int* o = out + a * 10;
    o[0] = s.calls;
    o[1] = s.early;
    o[2] = s.runs;
    o[3] = s.tcg_iters;
    for (int k = 0; k < 5; ++k) o[4 + k] = s.status[k];
    o[9] = s.gave_up;
  }
}

void dpgo_cpu_rbcd_status(void* h, double* rel, int* ready) {
  auto* E = static_cast<CpuEngine*>(h);
  for (int a = 0; a < E->K; ++a) {
    rel[a] = E->ag[a].status_rel;
    ready[a] = E->ag[a].ready;
  }
}

int dpgo_cpu_rbcd_color(void* h, int agent) { return static_cast<CpuEngine*>(h)->color[agent]; }

// Bounded timing sample (bench.py's cpu_baseline of the exact-preconditioner legs): the listed agents, OpenMP over
// them with `threads` threads, each first factorised (if its Q has no factor yet) and then updated `reps` times as
// selected agents (iterate(true) at the current Nesterov coefficients, neighbours' poses fixed).  factor_sec /
// update_sec [count]: per agent wall seconds of the factorisation and of one update (mean of reps).  Returns the wall
// seconds of the update phase (after every listed agent's factor is in place).
double dpgo_cpu_rbcd_time_sample(void* h, const int* agents, int count, int threads, int reps, double* factor_sec,
                                 double* update_sec) {
  auto* E = static_cast<CpuEngine*>(h);
  const int T = std::max(1, std::min(threads, static_cast<int>(E->work.size())));
#pragma omp parallel for num_threads(T) schedule(dynamic)
  for (int q = 0; q < count; ++q) {
    CpuAgent& c = E->ag[agents[q]];
    const double before = c.factor_sec;
    ensure_factor(c);
    factor_sec[q] = c.factor_sec - before;
  }
  const auto t0 = std::chrono::steady_clock::now();
#pragma omp parallel for num_threads(T) schedule(dynamic)
  for (int q = 0; q < count; ++q) {
    const auto u0 = std::chrono::steady_clock::now();
    for (int k = 0; k < reps; ++k) iterate_agent(*E, agents[q], true, false, E->work[omp_get_thread_num()]);
    update_sec[q] = std::chrono::duration<double>(std::chrono::steady_clock::now() - u0).count() / std::max(reps, 1);
  }
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// per agent: factorisations of the exact preconditioner and their total wall seconds
void dpgo_cpu_rbcd_factor_info(void* h, int* count, double* sec) {
  auto* E = static_cast<CpuEngine*>(h);
  for (int a = 0; a < E->K; ++a) {
    count[a] = E->ag[a].factor_count;
    sec[a] = E->ag[a].factor_sec;
  }
}
int dpgo_cpu_max_threads(void) { return omp_get_max_threads(); }

}  // extern "C"

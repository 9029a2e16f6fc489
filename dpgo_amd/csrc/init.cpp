// Chordal initialisation (chordalInitialization, src/DPGO_utils.cpp:377-424; used by
// PGOAgent::localInitialization for the L2 cost, src/PGOAgent.cpp:947-962, and by
// examples/MultiRobotExample.cpp:158).  The reference solves the two linear least-squares problems
// with SPQR; here their normal equations -- a d x d block connection Laplacian for the rotations
// (R_0 = I fixed) and a scalar graph Laplacian for the translations (t_0 = 0) -- are solved either by
// the host block Cholesky (chol.cpp, exact) or, for graphs whose factor would not fit (10^6-pose 3D
// grids: the top separator alone is a dense 3*10^4 square), by Jacobi-preconditioned CG on the GPU to
// a relative residual tolerance.  Same unique minimiser (connected graph); rotations are projected to
// SO(d) as projectToRotationGroup (:478-492).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "chol_internal.h"
#include "graph_internal.h"

namespace dpgo {

namespace {

// Symmetric block-sparse system over free poses, rows sorted by column with duplicates merged:
// block (j, col[k]) row-major bs x bs.  Assembled in O(entries) by counting, not by maps (the
// device path runs 10^6-pose graphs).
struct BlockSys {
  int n = 0, bs = 0;
  std::vector<int> rowptr, col;
  std::vector<double> blk;
};

// Edge list of the system: per edge its two free rows (-1 = the fixed anchor) and per edge the blocks
// Bii (row i), Bjj (row j), Bij (i, j) -- Bji = Bij^T.
struct SysBuilder {
  int n, bs;
  std::vector<int> ei, ej;
  std::vector<double> bii, bjj, bij;
  SysBuilder(int n_, int bs_) : n(n_), bs(bs_) {}
  void add(int i, int j, const double* Bii, const double* Bjj, const double* Bij) {
    const int b2 = bs * bs;
    ei.push_back(i);
    ej.push_back(j);
    bii.insert(bii.end(), Bii, Bii + b2);
    bjj.insert(bjj.end(), Bjj, Bjj + b2);
    bij.insert(bij.end(), Bij, Bij + b2);
  }
  void build(BlockSys& S) const {
    const int b2 = bs * bs;
    const size_t m = ei.size();
    S.n = n;
    S.bs = bs;
    std::vector<int> cnt(n + 1, 0);
    for (int j = 0; j < n; ++j) cnt[j + 1] = 1;  // diagonal
    for (size_t e = 0; e < m; ++e)
      if (ei[e] >= 0 && ej[e] >= 0) {
        ++cnt[ei[e] + 1];
        ++cnt[ej[e] + 1];
      }
    for (int j = 0; j < n; ++j) cnt[j + 1] += cnt[j];
    std::vector<int> c(cnt[n]);
    std::vector<double> b(static_cast<size_t>(cnt[n]) * b2, 0.0);
    std::vector<int> fill(cnt.begin(), cnt.end() - 1);
    for (int j = 0; j < n; ++j) c[fill[j]++] = j;
    for (size_t e = 0; e < m; ++e) {
      const int i = ei[e], j = ej[e];
      if (i >= 0) {  // diagonal of row i: first entry of the row, summed in edge order
        double* D = &b[static_cast<size_t>(cnt[i]) * b2];
        for (int x = 0; x < b2; ++x) D[x] += bii[e * b2 + x];
      }
      if (j >= 0) {
        double* D = &b[static_cast<size_t>(cnt[j]) * b2];
        for (int x = 0; x < b2; ++x) D[x] += bjj[e * b2 + x];
      }
      if (i >= 0 && j >= 0) {
        const int ki = fill[i]++, kj = fill[j]++;
        c[ki] = j;
        c[kj] = i;
        for (int u = 0; u < bs; ++u)
          for (int v = 0; v < bs; ++v) {
            b[static_cast<size_t>(ki) * b2 + u * bs + v] = bij[e * b2 + u * bs + v];
            b[static_cast<size_t>(kj) * b2 + v * bs + u] = bij[e * b2 + u * bs + v];
          }
      }
    }
    // sort each row by column and merge repeated (i, j) pairs (duplicate measurements)
    S.rowptr.assign(n + 1, 0);
    S.col.clear();
    S.blk.clear();
    S.col.reserve(c.size());
    S.blk.reserve(b.size());
    std::vector<int> idx;
    for (int j = 0; j < n; ++j) {
      idx.resize(cnt[j + 1] - cnt[j]);
      for (size_t x = 0; x < idx.size(); ++x) idx[x] = cnt[j] + static_cast<int>(x);
      std::stable_sort(idx.begin(), idx.end(), [&](int a, int bb) { return c[a] < c[bb]; });
      for (size_t x = 0; x < idx.size(); ++x) {
        const int k = idx[x];
        if (!S.col.empty() && static_cast<int>(S.col.size()) > S.rowptr[j] && S.col.back() == c[k]) {
          double* dst = &S.blk[S.blk.size() - b2];
          for (int y = 0; y < b2; ++y) dst[y] += b[static_cast<size_t>(k) * b2 + y];
        } else {
          S.col.push_back(c[k]);
          S.blk.insert(S.blk.end(), &b[static_cast<size_t>(k) * b2], &b[static_cast<size_t>(k) * b2] + b2);
        }
      }
      S.rowptr[j + 1] = static_cast<int>(S.col.size());
    }
  }
};

// Direct solve with the host supernodal Cholesky (blocks handed over column-major); rhs [row][bs][nr]
int solve_direct(const BlockSys& S, int nr, std::vector<double>& rhs_x, std::string& err);

// projectToRotationGroup (src/DPGO_utils.cpp:478-492) of a d x d row-major matrix: U V^T from a
// one-sided Jacobi SVD; if det(U) det(V) < 0 the column of U with the smallest singular value
// flips (Eigen's JacobiSVD sorts them descending and flips the last).
void project_rotation(int d, const double* M, double* out) {
  double W[3][3], V[3][3];
  for (int a = 0; a < d; ++a)
    for (int c = 0; c < d; ++c) {
      W[a][c] = M[a * d + c];
      V[a][c] = a == c ? 1.0 : 0.0;
    }
  for (int sweep = 0; sweep < 60; ++sweep) {
    bool rot = false;
    for (int p = 0; p < d - 1; ++p)
      for (int q = p + 1; q < d; ++q) {
        double al = 0, be = 0, ga = 0;
        for (int a = 0; a < d; ++a) {
          al += W[a][p] * W[a][p];
          be += W[a][q] * W[a][q];
          ga += W[a][p] * W[a][q];
        }
        if (std::fabs(ga) <= 1e-17 * std::sqrt(al * be) || ga == 0.0) continue;
        rot = true;
        const double zeta = (be - al) / (2 * ga);
        const double t = std::copysign(1.0, zeta) / (std::fabs(zeta) + std::sqrt(1 + zeta * zeta));
        const double c = 1 / std::sqrt(1 + t * t), s = c * t;
        for (int a = 0; a < d; ++a) {
          const double wp = W[a][p], wq = W[a][q];
          W[a][p] = c * wp - s * wq;
          W[a][q] = s * wp + c * wq;
          const double vp = V[a][p], vq = V[a][q];
          V[a][p] = c * vp - s * vq;
          V[a][q] = s * vp + c * vq;
        }
      }
    if (!rot) break;
  }
  double sig[3];
  int cmin = 0;
  for (int c = 0; c < d; ++c) {
    double s = 0;
    for (int a = 0; a < d; ++a) s += W[a][c] * W[a][c];
    sig[c] = std::sqrt(s);
    for (int a = 0; a < d; ++a) W[a][c] = sig[c] > 0 ? W[a][c] / sig[c] : 0.0;
    if (sig[c] < sig[cmin]) cmin = c;
  }
  auto det = [&](double (&A)[3][3]) {
    return d == 2 ? A[0][0] * A[1][1] - A[0][1] * A[1][0]
                  : A[0][0] * (A[1][1] * A[2][2] - A[1][2] * A[2][1]) - A[0][1] * (A[1][0] * A[2][2] - A[1][2] * A[2][0]) +
                        A[0][2] * (A[1][0] * A[2][1] - A[1][1] * A[2][0]);
  };
  if (det(W) * det(V) < 0)
    for (int a = 0; a < d; ++a) W[a][cmin] = -W[a][cmin];
  for (int a = 0; a < d; ++a)
    for (int c = 0; c < d; ++c) {
      double s = 0;
      for (int k = 0; k < d; ++k) s += W[a][k] * V[c][k];
      out[a * d + c] = s;
    }
}

int solve_direct(const BlockSys& S, int nr, std::vector<double>& rhs_x, std::string& err) {
  const int bs = S.bs, b2 = bs * bs, n = S.n;
  std::vector<double> cm(S.blk.size());
  for (size_t k = 0; k < S.col.size(); ++k)
    for (int u = 0; u < bs; ++u)
      for (int v = 0; v < bs; ++v) cm[k * b2 + v * bs + u] = S.blk[k * b2 + u * bs + v];
  SupernodalFactor L;
  if (supernodal_cholesky(n, bs, S.rowptr, S.col, cm, 0.0, 1L << 31, L, err) != 0) return -1;
  for (int a = 0; a < nr; ++a) {
    std::vector<double> x(static_cast<size_t>(n) * bs);
    for (int p = 0; p < n; ++p)
      for (int v = 0; v < bs; ++v) x[static_cast<size_t>(p) * bs + v] = rhs_x[(static_cast<size_t>(p) * bs + v) * nr + a];
    supernodal_solve(L, x);
    for (int p = 0; p < n; ++p)
      for (int v = 0; v < bs; ++v) rhs_x[(static_cast<size_t>(p) * bs + v) * nr + a] = x[static_cast<size_t>(p) * bs + v];
  }
  return 0;
}

// Jacobi-PCG on the device (one independent CG per right-hand side, advanced together): stops when
// every right-hand side's |r| <= rtol |b| or after max_iters iterations.
struct PcgReport {
  int iters = 0;
  double relres = 0.0;
};

int solve_pcg(const BlockSys& S, int nr, std::vector<double>& rhs_x, double rtol, int max_iters, PcgReport& rep,
              std::string& err) {
  const int bs = S.bs, b2 = bs * bs, n = S.n;
  const size_t L = static_cast<size_t>(n) * bs * nr;
  // block-Jacobi: inverse of each row's diagonal block (Gauss-Jordan, partial pivoting)
  std::vector<double> minv(static_cast<size_t>(n) * b2, 0.0);
  for (int j = 0; j < n; ++j) {
    double A[3][6] = {{0}};
    for (int k = S.rowptr[j]; k < S.rowptr[j + 1]; ++k)
      if (S.col[k] == j)
        for (int u = 0; u < bs; ++u)
          for (int v = 0; v < bs; ++v) A[u][v] = S.blk[static_cast<size_t>(k) * b2 + u * bs + v];
    for (int u = 0; u < bs; ++u) A[u][bs + u] = 1.0;
    for (int c = 0; c < bs; ++c) {
      int piv = c;
      for (int u = c + 1; u < bs; ++u)
        if (std::fabs(A[u][c]) > std::fabs(A[piv][c])) piv = u;
      for (int v = 0; v < 2 * bs; ++v) std::swap(A[c][v], A[piv][v]);
      if (A[c][c] == 0.0) {
        err = "singular diagonal block (is the pose graph connected?)";
        return -1;
      }
      const double inv = 1.0 / A[c][c];
      for (int v = 0; v < 2 * bs; ++v) A[c][v] *= inv;
      for (int u = 0; u < bs; ++u)
        if (u != c) {
          const double f = A[u][c];
          for (int v = 0; v < 2 * bs; ++v) A[u][v] -= f * A[c][v];
        }
    }
    for (int u = 0; u < bs; ++u)
      for (int v = 0; v < bs; ++v) minv[static_cast<size_t>(j) * b2 + u * bs + v] = A[u][bs + v];
  }
  hipStream_t st = nullptr;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
    err = "stream create failed";
    return -1;
  }
  struct StreamGuard {
    hipStream_t s;
    ~StreamGuard() {
      (void)hipStreamSynchronize(s);
      (void)hipStreamDestroy(s);
    }
  } guard{st};
  DevBuf<int> drp, dcol;
  DevBuf<double> dblk, dminv, x, r, z, pv, q, part;
  const int P2 = kPcgBlocks * 2 * nr;
  auto bad = [&](hipError_t e) {
    if (e == hipSuccess) return false;
    err = std::string("device: ") + hipGetErrorString(e);
    return true;
  };
  if (bad(drp.ensure(n + 1)) || bad(dcol.ensure(S.col.size())) || bad(dblk.ensure(S.blk.size())) ||
      bad(dminv.ensure(minv.size())) || bad(x.ensure(L)) || bad(r.ensure(L)) || bad(z.ensure(L)) ||
      bad(pv.ensure(L)) || bad(q.ensure(L)) || bad(part.ensure(P2)))
    return -1;
  if (bad(hipMemcpyAsync(drp.p, S.rowptr.data(), sizeof(int) * (n + 1), hipMemcpyHostToDevice, st)) ||
      bad(hipMemcpyAsync(dcol.p, S.col.data(), sizeof(int) * S.col.size(), hipMemcpyHostToDevice, st)) ||
      bad(hipMemcpyAsync(dblk.p, S.blk.data(), sizeof(double) * S.blk.size(), hipMemcpyHostToDevice, st)) ||
      bad(hipMemcpyAsync(dminv.p, minv.data(), sizeof(double) * minv.size(), hipMemcpyHostToDevice, st)) ||
      bad(hipMemcpyAsync(r.p, rhs_x.data(), sizeof(double) * L, hipMemcpyHostToDevice, st)) ||
      bad(hipMemsetAsync(x.p, 0, sizeof(double) * L, st)) || bad(hipMemsetAsync(q.p, 0, sizeof(double) * L, st)) ||
      bad(hipMemsetAsync(pv.p, 0, sizeof(double) * L, st)))
    return -1;
  std::vector<double> hp(P2);
  auto sums = [&](int q2, std::vector<double>& out) -> bool {  // fixed-order host sum of the partials
    if (bad(hipMemcpyAsync(hp.data(), part.p, sizeof(double) * kPcgBlocks * q2, hipMemcpyDeviceToHost, st)) ||
        bad(hipStreamSynchronize(st)))
      return false;
    out.assign(q2, 0.0);
    for (int g = 0; g < kPcgBlocks; ++g)
      for (int a = 0; a < q2; ++a) out[a] += hp[static_cast<size_t>(g) * q2 + a];
    return true;
  };
  PcgCoef zero{{0.0, 0.0, 0.0}};
  // x = 0, r = b: z = Minv r and <r, z>, |r|^2 (the update with alpha = 0); p = z
  if (bad(launch_pcg_update(bs, nr, n, zero, pv.p, q.p, x.p, r.p, z.p, dminv.p, part.p, st))) return -1;
  std::vector<double> s2, rz(nr), bn(nr);
  if (!sums(2 * nr, s2)) return -1;
  for (int a = 0; a < nr; ++a) {
    rz[a] = s2[a];
    bn[a] = std::sqrt(s2[nr + a]);
  }
  if (bad(launch_pcg_dir(bs, nr, n, zero, z.p, pv.p, st))) return -1;
  rep.iters = 0;
  rep.relres = 0.0;
  for (int a = 0; a < nr; ++a) rep.relres = std::max(rep.relres, bn[a] > 0 ? 1.0 : 0.0);
  while (rep.relres > rtol && rep.iters < max_iters) {
    if (bad(launch_pcg_spmv(bs, nr, n, drp.p, dcol.p, dblk.p, pv.p, q.p, st)) ||
        bad(launch_pcg_dot(bs, nr, n, pv.p, q.p, part.p, st)))
      return -1;
    std::vector<double> pq;
    if (!sums(nr, pq)) return -1;
    PcgCoef al = zero;
    for (int a = 0; a < nr; ++a) al.v[a] = (bn[a] > 0 && pq[a] != 0.0) ? rz[a] / pq[a] : 0.0;
    if (bad(launch_pcg_update(bs, nr, n, al, pv.p, q.p, x.p, r.p, z.p, dminv.p, part.p, st))) return -1;
    if (!sums(2 * nr, s2)) return -1;
    PcgCoef be = zero;
    rep.relres = 0.0;
    for (int a = 0; a < nr; ++a) {
      if (bn[a] > 0) rep.relres = std::max(rep.relres, std::sqrt(s2[nr + a]) / bn[a]);
      be.v[a] = (bn[a] > 0 && rz[a] != 0.0) ? s2[a] / rz[a] : 0.0;
      rz[a] = s2[a];
    }
    ++rep.iters;
    if (bad(launch_pcg_dir(bs, nr, n, be, z.p, pv.p, st))) return -1;
  }
  if (bad(hipMemcpyAsync(rhs_x.data(), x.p, sizeof(double) * L, hipMemcpyDeviceToHost, st)) || bad(hipStreamSynchronize(st)))
    return -1;
  if (!(rep.relres <= rtol)) {
    err = "PCG did not reach the tolerance (relative residual " + std::to_string(rep.relres) + " after " +
          std::to_string(rep.iters) + " iterations)";
    return -1;
  }
  return 0;
}

// chordalInitialization with the linear solves done by `solve`: rotations (d x d block connection
// Laplacian, d right-hand sides = the rows of R) then translations (scalar Laplacian, d right-hand
// sides), as the two SPQR solves of the reference (:377-476).  The poses flagged in `anchor` are held
// at R = I, t = 0 (the reference: pose 0 only); each connected component needs one.
template <typename Solver>
int chordal_core(int d, int n, int m, const int* p1, const int* p2, const double* R, const double* t,
                 const double* kappa, const double* tau, const std::vector<char>& anchor, double* T_out,
                 Solver&& solve, std::string& err) {
  if (n < 1) {
    err = "chordal initialisation: no poses";
    return -1;
  }
  const int d2 = d * d;
  std::vector<int> row(n, -1);
  int nf = 0;
  for (int p = 0; p < n; ++p)
    if (!anchor[p]) row[p] = nf++;
  std::vector<double> Rch(static_cast<size_t>(n) * d2, 0.0);  // R_i row-major per pose
  for (int p = 0; p < n; ++p)
    for (int u = 0; u < d; ++u) Rch[static_cast<size_t>(p) * d2 + u * d + u] = 1.0;
  if (nf > 0) {
    // ---- rotations: min sum kappa |R_j - R_i R_ij|_F^2; the rows of R decouple into d right-hand
    // sides.  x A x^T form: A_ii += k R R^T, A_jj += k I, A_ij = -k R
    SysBuilder B(nf, d);
    std::vector<double> rhs(static_cast<size_t>(nf) * d * d, 0.0);  // [row][v][row a of R]
    double Bii[9], Bjj[9], Bij[9];
    for (int e = 0; e < m; ++e) {
      const int i = p1[e], j = p2[e], ri = row[i], rj = row[j];
      if (ri < 0 && rj < 0) continue;
      const double k = kappa[e];
      const double* Re = R + static_cast<size_t>(e) * d2;
      for (int u = 0; u < d; ++u)
        for (int v = 0; v < d; ++v) {
          double s = 0;
          for (int w = 0; w < d; ++w) s += Re[u * d + w] * Re[v * d + w];
          Bii[u * d + v] = k * s;
          Bjj[u * d + v] = u == v ? k : 0.0;
          Bij[u * d + v] = -k * Re[u * d + v];
        }
      B.add(ri, rj, Bii, Bjj, Bij);
      if (ri < 0) {  // fixed x_i = row a of I: rhs_j -= x_i A_ij = k (row a of R)
        for (int a = 0; a < d; ++a)
          for (int v = 0; v < d; ++v) rhs[(static_cast<size_t>(rj) * d + v) * d + a] += k * Re[a * d + v];
      } else if (rj < 0) {  // rhs_i -= x_j A_ji, A_ji = -k R^T  -> += k R(:, a)
        for (int a = 0; a < d; ++a)
          for (int v = 0; v < d; ++v) rhs[(static_cast<size_t>(ri) * d + v) * d + a] += k * Re[v * d + a];
      }
    }
    BlockSys S;
    B.build(S);
    if (solve(S, d, rhs, err) != 0) {
      err = "chordal initialisation (rotations): " + err + " (is the pose graph connected?)";
      return -1;
    }
    for (int p = 0; p < n; ++p) {
      if (row[p] < 0) continue;
      double M[9], P[9];
      for (int a = 0; a < d; ++a)
        for (int v = 0; v < d; ++v) M[a * d + v] = rhs[(static_cast<size_t>(row[p]) * d + v) * d + a];
      project_rotation(d, M, P);
      std::memcpy(&Rch[static_cast<size_t>(p) * d2], P, sizeof(double) * d2);
    }
  }
  // ---- translations (recoverTranslations): min sum tau |t_j - t_i - R_i t_ij|^2, anchors t = 0
  std::vector<double> tt(static_cast<size_t>(n) * d, 0.0);
  if (nf > 0) {
    SysBuilder B(nf, 1);
    std::vector<double> rhs(static_cast<size_t>(nf) * d, 0.0);  // [row][component]
    for (int e = 0; e < m; ++e) {
      const int i = p1[e], j = p2[e], ri = row[i], rj = row[j];
      if (ri < 0 && rj < 0) continue;
      const double w = tau[e], mw = -w;
      double c[3] = {0, 0, 0};  // R_i t_ij
      for (int u = 0; u < d; ++u)
        for (int v = 0; v < d; ++v) c[u] += Rch[static_cast<size_t>(i) * d2 + u * d + v] * t[static_cast<size_t>(e) * d + v];
      B.add(ri, rj, &w, &w, &mw);
      for (int u = 0; u < d; ++u) {
        if (rj >= 0) rhs[static_cast<size_t>(rj) * d + u] += w * c[u];
        if (ri >= 0) rhs[static_cast<size_t>(ri) * d + u] -= w * c[u];
      }
    }
    BlockSys S;
    B.build(S);
    if (solve(S, d, rhs, err) != 0) {
      err = "chordal initialisation (translations): " + err + " (is the pose graph connected?)";
      return -1;
    }
    for (int p = 0; p < n; ++p)
      if (row[p] >= 0)
        for (int u = 0; u < d; ++u) tt[static_cast<size_t>(p) * d + u] = rhs[static_cast<size_t>(row[p]) * d + u];
  }
  // ---- T = [R_i | t_i] per pose, d x (d+1) n column-major
  const int b = d + 1;
  for (int p = 0; p < n; ++p)
    for (int c = 0; c < b; ++c)
      for (int u = 0; u < d; ++u)
        T_out[(static_cast<size_t>(p) * b + c) * d + u] =
            c < d ? Rch[static_cast<size_t>(p) * d2 + u * d + c] : tt[static_cast<size_t>(p) * d + u];
  return 0;
}

// Breadth-first eccentricity centre of the pose set `verts` (edges restricted to it): the middle of
// a longest BFS path found by two sweeps (exact on trees, within one hop of the centre on grids).
int bfs_centre(const std::vector<std::vector<int>>& adj, const std::vector<int>& verts, const std::vector<int>& agent_of,
               int a, std::vector<int>& dist, std::vector<int>& par) {
  auto sweep = [&](int s) {
    std::vector<int> q{s};
    dist[s] = 0;
    par[s] = -1;
    int last = s;
    for (size_t h = 0; h < q.size(); ++h) {
      const int v = q[h];
      last = v;
      for (int u : adj[v])
        if (agent_of[u] == a && dist[u] < 0) {
          dist[u] = dist[v] + 1;
          par[u] = v;
          q.push_back(u);
        }
    }
    for (int v : q) dist[v] = -1;
    return last;
  };
  const int x = sweep(verts[0]);
  const int y = sweep(x);  // par[] now describes BFS tree from x; path y -> x
  std::vector<int> path;
  for (int v = y; v >= 0; v = par[v]) path.push_back(v);
  return path[path.size() / 2];
}

}  // namespace

int chordal_initialization(int d, int n, int m, const int* p1, const int* p2, const double* R, const double* t,
                           const double* kappa, const double* tau, double* T_out, std::string& err) {
  std::vector<char> anchor(std::max(n, 1), 0);
  anchor[0] = 1;  // R_0 = I, t_0 = 0 (:389, :458)
  return chordal_core(d, n, m, p1, p2, R, t, kappa, tau, anchor, T_out,
                      [](const BlockSys& S, int nr, std::vector<double>& rx, std::string& e) {
                        return solve_direct(S, nr, rx, e);
                      },
                      err);
}

int chordal_initialization_gpu(int d, int n, int m, const int* p1, const int* p2, const double* R, const double* t,
                               const double* kappa, const double* tau, double* T_out, double rtol, int max_iters,
                               int* iters, double* relres, std::string& err) {
  int it_sum = 0;
  double rr = 0.0;
  std::vector<char> anchor(std::max(n, 1), 0);
  anchor[0] = 1;
  const int rc = chordal_core(d, n, m, p1, p2, R, t, kappa, tau, anchor, T_out,
                              [&](const BlockSys& S, int nr, std::vector<double>& rx, std::string& e) {
                                PcgReport rep;
                                const int r = solve_pcg(S, nr, rx, rtol, max_iters, rep, e);
                                it_sum += rep.iters;
                                rr = std::max(rr, rep.relres);
                                return r;
                              },
                              err);
  if (iters) *iters = it_sum;
  if (relres) *relres = rr;
  return rc;
}

int distributed_initialization(int d, int n, int m, const int* p1, const int* p2, const double* R, const double* t,
                               const double* kappa, const double* tau, const int* agent_of, int num_agents, bool gpu,
                               double rtol, int max_iters, double* T_out, int* iters, double* relres,
                               std::string& err) {
  const int d2 = d * d, b = d + 1;
  // ---- PGOAgent::localInitialization: chordal on every agent's private graph (all agents in one
  // block-diagonal system; one anchor per agent, at the agent's BFS centre)
  std::vector<int> q1, q2;
  std::vector<double> qR, qt, qk, qtau;
  std::vector<std::vector<int>> adj(n);
  std::vector<std::vector<int>> verts(num_agents);
  for (int p = 0; p < n; ++p) verts[agent_of[p]].push_back(p);
  for (int e = 0; e < m; ++e) {
    const int i = p1[e], j = p2[e];
    if (agent_of[i] != agent_of[j]) continue;
    q1.push_back(i);
    q2.push_back(j);
    qR.insert(qR.end(), R + static_cast<size_t>(e) * d2, R + static_cast<size_t>(e + 1) * d2);
    qt.insert(qt.end(), t + static_cast<size_t>(e) * d, t + static_cast<size_t>(e + 1) * d);
    qk.push_back(kappa[e]);
    qtau.push_back(tau[e]);
    adj[i].push_back(j);
    adj[j].push_back(i);
  }
  std::vector<char> anchor(n, 0);
  {
    std::vector<int> dist(n, -1), par(n, -1);
    for (int a = 0; a < num_agents; ++a) {
      if (verts[a].empty()) {
        err = "agent without poses";
        return -1;
      }
      anchor[bfs_centre(adj, verts[a], std::vector<int>(agent_of, agent_of + n), a, dist, par)] = 1;
    }
  }
  std::vector<double> Tl(static_cast<size_t>(n) * d * b);
  int it_sum = 0;
  double rr = 0.0;
  auto direct = [](const BlockSys& S, int nr, std::vector<double>& rx, std::string& e) {
    return solve_direct(S, nr, rx, e);
  };
  auto pcg = [&](const BlockSys& S, int nr, std::vector<double>& rx, std::string& e) {
    PcgReport rep;
    const int r = solve_pcg(S, nr, rx, rtol, max_iters, rep, e);
    it_sum += rep.iters;
    rr = std::max(rr, rep.relres);
    return r;
  };
  const int mq = static_cast<int>(q1.size());
  const int rc = gpu ? chordal_core(d, n, mq, q1.data(), q2.data(), qR.data(), qt.data(), qk.data(), qtau.data(),
                                    anchor, Tl.data(), pcg, err)
                     : chordal_core(d, n, mq, q1.data(), q2.data(), qR.data(), qt.data(), qk.data(), qtau.data(),
                                    anchor, Tl.data(), direct, err);
  if (iters) *iters = it_sum;
  if (relres) *relres = rr;
  if (rc != 0) return rc;
  auto Rl = [&](int p, int u, int c) { return Tl[(static_cast<size_t>(p) * b + c) * d + u]; };  // R_loc(u, c)
  auto tl = [&](int p, int u) { return Tl[(static_cast<size_t>(p) * b + d) * d + u]; };
  // ---- initializeInGlobalFrame: agents join the frame of the agent holding pose 0 in breadth-first
  // order over the agent graph; each takes the L2 average, over its shared loop closures with agents
  // already in the frame, of the frame transform every closure implies (rotations: chordal mean
  // projected to SO(d); translations: tau-weighted mean).  The reference averages robustly (GNC-TLS,
  // robustSinglePoseAveraging); on outlier-free data the two coincide.
  std::vector<std::vector<int>> shared(num_agents);
  std::vector<std::set<int>> nbr(num_agents);
  for (int e = 0; e < m; ++e) {
    const int ai = agent_of[p1[e]], aj = agent_of[p2[e]];
    if (ai == aj) continue;
    shared[ai].push_back(e);
    shared[aj].push_back(e);
    nbr[ai].insert(aj);
    nbr[aj].insert(ai);
  }
  std::vector<double> FR(static_cast<size_t>(num_agents) * d2, 0.0), Ft(static_cast<size_t>(num_agents) * d, 0.0);
  std::vector<char> done(num_agents, 0);
  std::vector<int> order{agent_of[0]};
  done[agent_of[0]] = 1;
  for (int u = 0; u < d; ++u) FR[static_cast<size_t>(agent_of[0]) * d2 + u * d + u] = 1.0;
  // world pose of a pose of an aligned agent
  auto world = [&](int p, double* Rw, double* tw) {
    const int a = agent_of[p];
    const double* F = &FR[static_cast<size_t>(a) * d2];
    for (int u = 0; u < d; ++u) {
      for (int c = 0; c < d; ++c) {
        double s = 0.0;
        for (int w = 0; w < d; ++w) s += F[u * d + w] * Rl(p, w, c);
        Rw[u * d + c] = s;
      }
      double s = Ft[static_cast<size_t>(a) * d + u];
      for (int w = 0; w < d; ++w) s += F[u * d + w] * tl(p, w);
      tw[u] = s;
    }
  };
  for (size_t h = 0; h < order.size(); ++h) {
    for (int A : nbr[order[h]]) {
      if (done[A]) continue;
      // closures of A to agents already in the frame: implied world pose of A's endpoint
      struct Est {
        int p;
        double Rw[9], tw[3], w, wk;
      };
      std::vector<Est> est;
      for (int e : shared[A]) {
        const int i = p1[e], j = p2[e];
        const bool a_is_j = agent_of[j] == A;
        const int other = a_is_j ? i : j;
        if (!done[agent_of[other]]) continue;
        double Ro[9], to[3];
        world(other, Ro, to);
        const double* Re = R + static_cast<size_t>(e) * d2;
        const double* te = t + static_cast<size_t>(e) * d;
        Est x;
        x.p = a_is_j ? j : i;
        x.w = tau[e];
        x.wk = kappa[e];
        for (int u = 0; u < d; ++u)
          for (int c = 0; c < d; ++c) {
            double s = 0.0;
            for (int w = 0; w < d; ++w) s += a_is_j ? Ro[u * d + w] * Re[w * d + c] : Ro[u * d + w] * Re[c * d + w];
            x.Rw[u * d + c] = s;  // T_j = T_i T_e, or T_i = T_j T_e^-1
          }
        for (int u = 0; u < d; ++u) {
          double s = 0.0;
          for (int w = 0; w < d; ++w) s += (a_is_j ? Ro[u * d + w] : x.Rw[u * d + w]) * te[w];
          x.tw[u] = a_is_j ? to[u] + s : to[u] - s;
        }
        est.push_back(x);
      }
      if (est.empty()) continue;
      // rotation: chordal mean of Rw R_loc^T (kappa-weighted) projected to SO(d)
      double M[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
      for (const auto& x : est) {
        const double k = x.wk;
        for (int u = 0; u < d; ++u)
          for (int c = 0; c < d; ++c) {
            double s = 0.0;
            for (int w = 0; w < d; ++w) s += x.Rw[u * d + w] * Rl(x.p, c, w);
            M[u * d + c] += k * s;
          }
      }
      double* F = &FR[static_cast<size_t>(A) * d2];
      project_rotation(d, M, F);
      double tsum[3] = {0, 0, 0}, wsum = 0.0;
      for (const auto& x : est) {
        for (int u = 0; u < d; ++u) {
          double s = 0.0;
          for (int w = 0; w < d; ++w) s += F[u * d + w] * tl(x.p, w);
          tsum[u] += x.w * (x.tw[u] - s);
        }
        wsum += x.w;
      }
      for (int u = 0; u < d; ++u) Ft[static_cast<size_t>(A) * d + u] = tsum[u] / wsum;
      done[A] = 1;
      order.push_back(A);
    }
  }
  for (int a = 0; a < num_agents; ++a)
    if (!done[a]) {
      err = "agent graph is not connected (an agent shares no loop closure with the others)";
      return -1;
    }
  for (int p = 0; p < n; ++p) {
    double Rw[9], tw[3];
    world(p, Rw, tw);
    for (int u = 0; u < d; ++u) {
      for (int c = 0; c < d; ++c) T_out[(static_cast<size_t>(p) * b + c) * d + u] = Rw[u * d + c];
      T_out[(static_cast<size_t>(p) * b + d) * d + u] = tw[u];
    }
  }
  return 0;
}

void project_to_rotation(int d, const double* M, double* out) { project_rotation(d, M, out); }

}  // namespace dpgo

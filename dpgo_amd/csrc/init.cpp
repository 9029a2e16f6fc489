// Chordal initialisation (chordalInitialization, src/DPGO_utils.cpp:377-424; used by
// PGOAgent::localInitialization for the L2 cost, src/PGOAgent.cpp:947-962).  The reference solves the
// two linear least-squares problems with SPQR; here their normal equations -- a d x d block
// connection Laplacian for the rotations (R_0 = I fixed) and a scalar graph Laplacian for the
// translations (t_0 = 0) -- are factorised by the host block Cholesky (chol.cpp).  Same unique
// minimiser (connected graph); rotations are projected to SO(d) as projectToRotationGroup
// (:478-492).  One-time host work, like the reference's.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "chol_internal.h"
#include "graph_internal.h"

namespace dpgo {

namespace {

// symmetric block matrix as BSR (block (j, i) column-major) from a map of row-major blocks
struct SymBlocks {
  int n, b;
  std::vector<std::map<int, std::vector<double>>> rows;
  SymBlocks(int n_, int b_) : n(n_), b(b_), rows(n_) {}
  double* at(int i, int j) {  // block (i, j), row-major
    auto& blk = rows[i][j];
    if (blk.empty()) blk.assign(static_cast<size_t>(b) * b, 0.0);
    return blk.data();
  }
  void to_bsr(std::vector<int>& rowptr, std::vector<int>& col, std::vector<double>& blocks) const {
    rowptr.assign(n + 1, 0);
    col.clear();
    blocks.clear();
    for (int j = 0; j < n; ++j) {
      for (const auto& [i, blk] : rows[j]) {  // block (j, i) row-major -> column-major
        col.push_back(i);
        for (int v = 0; v < b; ++v)
          for (int u = 0; u < b; ++u) blocks.push_back(blk[u * b + v]);
      }
      rowptr[j + 1] = static_cast<int>(col.size());
    }
  }
};

// Solve (L L^T) x = rhs in place; rhs indexed by the ORIGINAL pose order, b values per pose.
void chol_solve(const BlockCholesky& L, std::vector<double>& rhs) {
  const int n = L.n, b = L.b, bb = b * b;
  std::vector<double> y(static_cast<size_t>(n) * b);
  for (int j = 0; j < n; ++j)
    for (int u = 0; u < b; ++u) y[static_cast<size_t>(j) * b + u] = rhs[static_cast<size_t>(L.perm[j]) * b + u];
  for (int j = 0; j < n; ++j) {  // forward: L y = rhs, by columns
    const double* D = &L.blocks[static_cast<size_t>(L.colptr[j]) * bb];
    double* yj = &y[static_cast<size_t>(j) * b];
    for (int u = 0; u < b; ++u) {
      double s = yj[u];
      for (int w = 0; w < u; ++w) s -= D[u * b + w] * yj[w];
      yj[u] = s / D[u * b + u];
    }
    for (int p = L.colptr[j] + 1; p < L.colptr[j + 1]; ++p) {
      const double* Lij = &L.blocks[static_cast<size_t>(p) * bb];
      double* yi = &y[static_cast<size_t>(L.rowidx[p]) * b];
      for (int u = 0; u < b; ++u)
        for (int w = 0; w < b; ++w) yi[u] -= Lij[u * b + w] * yj[w];
    }
  }
  for (int j = n - 1; j >= 0; --j) {  // backward: L^T x = y
    double* yj = &y[static_cast<size_t>(j) * b];
    for (int p = L.colptr[j] + 1; p < L.colptr[j + 1]; ++p) {
      const double* Lij = &L.blocks[static_cast<size_t>(p) * bb];
      const double* xi = &y[static_cast<size_t>(L.rowidx[p]) * b];
      for (int w = 0; w < b; ++w)
        for (int u = 0; u < b; ++u) yj[w] -= Lij[u * b + w] * xi[u];
    }
    const double* D = &L.blocks[static_cast<size_t>(L.colptr[j]) * bb];
    for (int u = b - 1; u >= 0; --u) {
      double s = yj[u];
      for (int w = u + 1; w < b; ++w) s -= D[w * b + u] * yj[w];
      yj[u] = s / D[u * b + u];
    }
  }
  for (int j = 0; j < n; ++j)
    for (int u = 0; u < b; ++u) rhs[static_cast<size_t>(L.perm[j]) * b + u] = y[static_cast<size_t>(j) * b + u];
}

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

}  // namespace

int chordal_initialization(int d, int n, int m, const int* p1, const int* p2, const double* R, const double* t,
                           const double* kappa, const double* tau, double* T_out, std::string& err) {
  if (n < 1) {
    err = "chordal initialisation: no poses";
    return -1;
  }
  const int d2 = d * d, nf = n - 1;
  std::vector<double> Rch(static_cast<size_t>(n) * d2, 0.0);  // R_i row-major per pose
  for (int u = 0; u < d; ++u) Rch[u * d + u] = 1.0;
  if (nf > 0) {
    // ---- rotations: min sum kappa |R_j - R_i R_ij|_F^2, R_0 = I; rows of R decouple into d
    // right-hand sides of the d x d block connection Laplacian (free poses 1..n-1)
    SymBlocks Q(nf, d);
    std::vector<double> rhs(static_cast<size_t>(nf) * d * d, 0.0);  // [pose][u][row a]
    for (int e = 0; e < m; ++e) {
      const int i = p1[e], j = p2[e];
      const double k = kappa[e];
      const double* Re = R + static_cast<size_t>(e) * d2;
      // Q_ii += k R R^T, Q_jj += k I, Q_ij = -k R, Q_ji = -k R^T (x Q x^T with x = a row of R)
      if (i > 0) {
        double* B = Q.at(i - 1, i - 1);
        for (int u = 0; u < d; ++u)
          for (int v = 0; v < d; ++v) {
            double s = 0;
            for (int w = 0; w < d; ++w) s += Re[u * d + w] * Re[v * d + w];
            B[u * d + v] += k * s;
          }
      }
      if (j > 0) {
        double* B = Q.at(j - 1, j - 1);
        for (int u = 0; u < d; ++u) B[u * d + u] += k;
      }
      if (i > 0 && j > 0) {
        double* Bij = Q.at(i - 1, j - 1);
        double* Bji = Q.at(j - 1, i - 1);
        for (int u = 0; u < d; ++u)
          for (int v = 0; v < d; ++v) {
            Bij[u * d + v] -= k * Re[u * d + v];
            Bji[v * d + u] -= k * Re[u * d + v];
          }
      } else if (i == 0 && j > 0) {  // fixed x_0 = row a of I: rhs_j -= x_0 Q_0j = -k (row a of R)
        for (int a = 0; a < d; ++a)
          for (int v = 0; v < d; ++v) rhs[(static_cast<size_t>(j - 1) * d + v) * d + a] += k * Re[a * d + v];
      } else if (j == 0 && i > 0) {  // rhs_i -= x_0 Q_0i, Q_0i = -k R^T  -> += k (R^T row a) = k R(:, a)
        for (int a = 0; a < d; ++a)
          for (int v = 0; v < d; ++v) rhs[(static_cast<size_t>(i - 1) * d + v) * d + a] += k * Re[v * d + a];
      }
    }
    std::vector<int> rowptr, col;
    std::vector<double> blocks;
    Q.to_bsr(rowptr, col, blocks);
    BlockCholesky L;
    if (block_cholesky(nf, d, rowptr, col, blocks, 0.0, 200u * 1000u * 1000u, L, err) != 0) {
      err = "chordal initialisation (rotations): " + err + " (is the pose graph connected?)";
      return -1;
    }
    for (int a = 0; a < d; ++a) {
      std::vector<double> x(static_cast<size_t>(nf) * d);
      for (int p = 0; p < nf; ++p)
        for (int v = 0; v < d; ++v) x[static_cast<size_t>(p) * d + v] = rhs[(static_cast<size_t>(p) * d + v) * d + a];
      chol_solve(L, x);
      for (int p = 0; p < nf; ++p)
        for (int v = 0; v < d; ++v) Rch[static_cast<size_t>(p + 1) * d2 + a * d + v] = x[static_cast<size_t>(p) * d + v];
    }
    for (int p = 1; p < n; ++p) {
      double P[9];
      project_rotation(d, &Rch[static_cast<size_t>(p) * d2], P);
      std::memcpy(&Rch[static_cast<size_t>(p) * d2], P, sizeof(double) * d2);
    }
  }
  // ---- translations (recoverTranslations): min sum tau |t_j - t_i - R_i t_ij|^2, t_0 = 0
  std::vector<double> tt(static_cast<size_t>(n) * d, 0.0);
  if (nf > 0) {
    SymBlocks L1(nf, 1);
    std::vector<double> rhs(static_cast<size_t>(nf) * d, 0.0);  // [pose][component]
    for (int e = 0; e < m; ++e) {
      const int i = p1[e], j = p2[e];
      const double w = tau[e];
      double c[3] = {0, 0, 0};  // R_i t_ij
      for (int u = 0; u < d; ++u)
        for (int v = 0; v < d; ++v) c[u] += Rch[static_cast<size_t>(i) * d2 + u * d + v] * t[static_cast<size_t>(e) * d + v];
      if (i > 0) *L1.at(i - 1, i - 1) += w;
      if (j > 0) *L1.at(j - 1, j - 1) += w;
      if (i > 0 && j > 0) {
        *L1.at(i - 1, j - 1) -= w;
        *L1.at(j - 1, i - 1) -= w;
      }
      for (int u = 0; u < d; ++u) {
        if (j > 0) rhs[static_cast<size_t>(j - 1) * d + u] += w * c[u];
        if (i > 0) rhs[static_cast<size_t>(i - 1) * d + u] -= w * c[u];
      }
    }
    std::vector<int> rowptr, col;
    std::vector<double> blocks;
    L1.to_bsr(rowptr, col, blocks);
    BlockCholesky L;
    if (block_cholesky(nf, 1, rowptr, col, blocks, 0.0, 200u * 1000u * 1000u, L, err) != 0) {
      err = "chordal initialisation (translations): " + err + " (is the pose graph connected?)";
      return -1;
    }
    for (int u = 0; u < d; ++u) {
      std::vector<double> x(nf);
      for (int p = 0; p < nf; ++p) x[p] = rhs[static_cast<size_t>(p) * d + u];
      chol_solve(L, x);
      for (int p = 0; p < nf; ++p) tt[static_cast<size_t>(p + 1) * d + u] = x[p];
    }
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

}  // namespace dpgo

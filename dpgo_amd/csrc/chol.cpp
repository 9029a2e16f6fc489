// Host supernodal Cholesky of P = Q + shift I for the exact preconditioner (QuadraticProblem::setQ,
// src/QuadraticProblem.cpp:37-41 factorises Q + 0.1 I with CHOLMOD; PreConditioner :75-87 applies it).
// Built once per Q, on the host like the reference's factorisation; the per-iteration triangular
// solves run on the GPU as dense panel products, one launch per tree level (kernels.hip, k_sn_*).
//
// Ordering: recursive nested dissection of the pose graph (BFS level-structure separators); every
// separator, and every leaf part of at most kLeaf poses, is one supernode.  Numeric: multifrontal --
// per supernode a dense frontal matrix over S and its row structure R (the original entries of
// the S columns plus the children's update matrices), its dense Cholesky, and the update matrix
// F_RR - L_RS L_RS^T handed to the parent.  The result is exact up to rounding like CHOLMOD's (which
// orders and factorises differently, so bits differ but P^-1 v agrees to cond(P) * eps).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "chol_internal.h"

namespace dpgo {

namespace {

constexpr size_t kLeaf = 32;  // poses: a leaf part is factorised as one dense supernode

// BFS from s over the vertices with mark == tag: levels (vertex lists).
void bfs_levels(const std::vector<std::vector<int>>& adj, int s, const std::vector<int>& mark, int tag,
                std::vector<int>& level, std::vector<std::vector<int>>& levels) {
  levels.clear();
  std::vector<int> cur{s}, nxt;
  level[s] = 0;
  while (!cur.empty()) {
    levels.push_back(cur);
    nxt.clear();
    for (int v : cur)
      for (int u : adj[v])
        if (mark[u] == tag && level[u] < 0) {
          level[u] = static_cast<int>(levels.size());
          nxt.push_back(u);
        }
    cur.swap(nxt);
  }
}

struct TreeBuilder {
  const std::vector<std::vector<int>>& adj;
  std::vector<SnNode>& nodes;
  std::vector<int> mark, level;
  int next_tag = 0;

  TreeBuilder(const std::vector<std::vector<int>>& a, std::vector<SnNode>& out, int n)
      : adj(a), nodes(out), mark(n, -1), level(n, -1) {}

  int leaf(std::vector<int> verts, int depth) {
    std::sort(verts.begin(), verts.end(), [&](int x, int y) {
      return adj[x].size() != adj[y].size() ? adj[x].size() < adj[y].size() : x < y;
    });
    SnNode nd;
    nd.S = std::move(verts);
    nd.depth = depth;
    nodes.push_back(std::move(nd));
    return static_cast<int>(nodes.size()) - 1;
  }

  int join(std::vector<int> S, std::vector<int> children, int depth) {
    const int id = static_cast<int>(nodes.size());
    for (int c : children) nodes[c].parent = id;
    SnNode nd;
    nd.S = std::move(S);
    nd.children = std::move(children);
    nd.depth = depth;
    nodes.push_back(std::move(nd));
    return id;
  }

  // node of the part `verts` at `depth`; children are appended first (postorder)
  int build(std::vector<int> verts, int depth) {
    if (verts.size() <= kLeaf) return leaf(std::move(verts), depth);
    const int tag = next_tag++;
    for (int v : verts) {
      mark[v] = tag;
      level[v] = -1;
    }
    std::vector<std::vector<int>> comps, lv;
    for (int v : verts) {
      if (level[v] >= 0) continue;
      bfs_levels(adj, v, mark, tag, level, lv);
      std::vector<int> comp;
      for (auto& l : lv) comp.insert(comp.end(), l.begin(), l.end());
      comps.push_back(std::move(comp));
    }
    if (comps.size() > 1) {  // independent components: an empty supernode joins them
      std::vector<int> ch;
      for (auto& c : comps) ch.push_back(build(std::move(c), depth + 1));
      return join({}, std::move(ch), depth);
    }
    // pseudo-peripheral start: two sweeps
    for (int v : verts) level[v] = -1;
    bfs_levels(adj, verts[0], mark, tag, level, lv);
    const int far = lv.back().back();
    for (int v : verts) level[v] = -1;
    bfs_levels(adj, far, mark, tag, level, lv);
    if (lv.size() < 3) return leaf(std::move(verts), depth);  // no useful separator: one dense block
    // separator = the level that splits the vertex count most evenly (not an end level)
    size_t acc = 0, best = 1;
    for (size_t l = 0; l + 1 < lv.size(); ++l) {
      acc += lv[l].size();
      if (acc * 2 >= verts.size()) {
        best = std::max<size_t>(1, l);
        break;
      }
    }
    best = std::min(best, lv.size() - 2);
    std::vector<int> A, B, S = lv[best];
    for (size_t l = 0; l < lv.size(); ++l) {
      if (l == best) continue;
      auto& dst = l < best ? A : B;
      dst.insert(dst.end(), lv[l].begin(), lv[l].end());
    }
    const int ca = build(std::move(A), depth + 1);
    const int cb = build(std::move(B), depth + 1);
    std::sort(S.begin(), S.end());
    return join(std::move(S), {ca, cb}, depth);
  }
};

// ---- dense kernels on row-major storage (ld = leading dimension) ---------------------------------
double dot(const double* a, const double* b, int n) {
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  int k = 0;
  for (; k + 4 <= n; k += 4) {
    s0 += a[k] * b[k];
    s1 += a[k + 1] * b[k + 1];
    s2 += a[k + 2] * b[k + 2];
    s3 += a[k + 3] * b[k + 3];
  }
  for (; k < n; ++k) s0 += a[k] * b[k];
  return (s0 + s2) + (s1 + s3);
}

// lower Cholesky of the leading n x n block in place (upper part left untouched); false if not PD
bool potrf(double* A, int n, long ld) {
  for (int j = 0; j < n; ++j) {
    double* rj = A + j * ld;
    const double d = rj[j] - dot(rj, rj, j);
    if (!(d > 0.0)) return false;
    const double l = std::sqrt(d);
    rj[j] = l;
    const double inv = 1.0 / l;
    for (int i = j + 1; i < n; ++i) {
      double* ri = A + i * ld;
      ri[j] = (ri[j] - dot(ri, rj, j)) * inv;
    }
  }
  return true;
}

// rows X (m x n, ld) := X L^-T for lower L (n x n, ldl): each row solves x L^T = row
void trsm_right_lt(double* X, int m, int n, long ld, const double* L, long ldl) {
  std::vector<double> inv(n);
  for (int j = 0; j < n; ++j) inv[j] = 1.0 / L[j * ldl + j];
  for (int i = 0; i < m; ++i) {
    double* x = X + i * ld;
    for (int j = 0; j < n; ++j) x[j] = (x[j] - dot(x, L + j * ldl, j)) * inv[j];
  }
}

// C (m x m lower, ldc) -= A A^T for A (m x k, lda), then mirrored to the upper triangle
void syrk_sub(double* C, long ldc, const double* A, int m, int k, long lda) {
  for (int i = 0; i < m; ++i)
    for (int j = 0; j <= i; ++j) C[i * ldc + j] -= dot(A + i * lda, A + j * lda, k);
  for (int i = 0; i < m; ++i)
    for (int j = i + 1; j < m; ++j) C[i * ldc + j] = C[j * ldc + i];
}

// Linv (n x n, row-major, lower) = L^-1 for lower L (ldl)
void trtri_lower(const double* L, int n, long ldl, double* Linv) {
  std::fill(Linv, Linv + static_cast<long>(n) * n, 0.0);
  std::vector<double> x(n);
  for (int c = 0; c < n; ++c) {  // column c: L x = e_c, x[i] = 0 for i < c
    std::fill(x.begin(), x.end(), 0.0);
    x[c] = 1.0 / L[c * ldl + c];
    for (int i = c + 1; i < n; ++i) {
      const double* li = L + i * ldl;
      x[i] = -dot(li + c, x.data() + c, i - c) / li[i];
    }
    for (int i = c; i < n; ++i) Linv[static_cast<long>(i) * n + c] = x[i];
  }
}

// M (m x n) = A (m x n, lda) Linv (n x n lower, row-major)
void trmm_right_lower(const double* A, int m, int n, long lda, const double* Linv, double* M) {
  for (int i = 0; i < m; ++i) {
    double* mi = M + static_cast<long>(i) * n;
    std::fill(mi, mi + n, 0.0);
    const double* ai = A + i * lda;
    for (int k = 0; k < n; ++k) {
      const double a = ai[k];
      if (a == 0.0) continue;
      const double* lk = Linv + static_cast<long>(k) * n;
      for (int j = 0; j <= k; ++j) mi[j] += a * lk[j];
    }
  }
}

}  // namespace

int supernodal_symbolic(int n, int b, const std::vector<int>& rowptr, const std::vector<int>& col, long max_doubles,
                        SupernodalFactor& F, std::string& err) {
  F = SupernodalFactor{};
  F.n = n;
  F.b = b;
  if (n == 0) return 0;
  // ---- ordering / tree on the pose graph
  std::vector<std::vector<int>> adj(n);
  for (int j = 0; j < n; ++j)
    for (int k = rowptr[j]; k < rowptr[j + 1]; ++k)
      if (col[k] != j) adj[j].push_back(col[k]);
  for (auto& a : adj) {
    std::sort(a.begin(), a.end());
    a.erase(std::unique(a.begin(), a.end()), a.end());
  }
  {
    std::vector<int> all(n);
    std::iota(all.begin(), all.end(), 0);
    TreeBuilder tb(adj, F.nodes, n);
    tb.build(std::move(all), 0);
  }
  auto& nodes = F.nodes;
  const int nn = static_cast<int>(nodes.size());
  // ---- symbolic: owner node of every pose, subtree ranges (postorder: [first[x], x]), row structures
  std::vector<int> owner(n, -1), first(nn), elim(n, 0);
  {
    int e = 0;
    for (int x = 0; x < nn; ++x) {
      first[x] = x;
      for (int c : nodes[x].children) first[x] = std::min(first[x], first[c]);
      for (int v : nodes[x].S) {
        owner[v] = x;
        elim[v] = e++;
      }
    }
  }
  std::vector<int> seen(n, -1);
  long total = 0;
  for (int x = 0; x < nn; ++x) {
    SnNode& nd = nodes[x];
    auto in_subtree = [&](int v) { return owner[v] >= first[x] && owner[v] <= x; };
    std::vector<int> R;
    auto add = [&](int v) {
      if (seen[v] != x && !in_subtree(v)) {
        seen[v] = x;
        R.push_back(v);
      }
    };
    for (int v : nd.S)
      for (int u : adj[v]) add(u);
    for (int c : nd.children)
      for (int u : nodes[c].R) add(u);
    std::sort(R.begin(), R.end(), [&](int p, int q) { return elim[p] < elim[q]; });
    nd.R = std::move(R);
    const long node_doubles =
        sn_panel_tiles(static_cast<int>(nd.S.size()) * b, static_cast<int>(nd.R.size()) * b) * kSnTile * kSnTile;
    if (node_doubles * 8 >= (1L << 32)) {  // the solves address a node's panel with 32-bit buffer offsets
      err = "exact preconditioner: one supernode's panel would exceed 4 GiB (use DPGO_PRECON_BLOCK_JACOBI)";
      return -1;
    }
    total += node_doubles;
    if (total > max_doubles) {
      err = "exact preconditioner: the supernodal factor panels of Q + 0.1 I would exceed " +
            std::to_string(max_doubles / (1L << 27)) + " GiB (use DPGO_PRECON_BLOCK_JACOBI for this size)";
      return -1;
    }
  }
  F.panel_doubles = total;
  // extend-add maps: child R -> parent frontal position
  std::vector<int> fpos(n, -1);
  for (int x = 0; x < nn; ++x) {
    const SnNode& nd = nodes[x];
    const int s = static_cast<int>(nd.S.size());
    for (int p = 0; p < s; ++p) fpos[nd.S[p]] = p;
    for (size_t q = 0; q < nd.R.size(); ++q) fpos[nd.R[q]] = s + static_cast<int>(q);
    for (int c : nd.children) {
      SnNode& ch = nodes[c];
      ch.to_parent.resize(ch.R.size());
      for (size_t i = 0; i < ch.R.size(); ++i) ch.to_parent[i] = fpos[ch.R[i]];
    }
    for (int v : nd.S) fpos[v] = -1;
    for (int v : nd.R) fpos[v] = -1;
  }
  return 0;
}

int supernodal_cholesky(int n, int b, const std::vector<int>& rowptr, const std::vector<int>& col,
                        const std::vector<double>& blocks_colmajor, double shift, long max_doubles,
                        SupernodalFactor& F, std::string& err) {
  const int bb = b * b;
  if (const int rc = supernodal_symbolic(n, b, rowptr, col, max_doubles, F, err)) return rc;
  if (n == 0) return 0;
  auto& nodes = F.nodes;
  const int nn = static_cast<int>(nodes.size());
  std::vector<int> fpos(n, -1);
  // ---- numeric, multifrontal in postorder
  std::vector<std::vector<double>> upd(nn);  // update matrices waiting for their parent
  std::vector<double> Fm, Linv, M;
  for (int x = 0; x < nn; ++x) {
    SnNode& nd = nodes[x];
    const int s = static_cast<int>(nd.S.size()), t = static_cast<int>(nd.R.size());
    const int sb = s * b, tb = t * b, m = sb + tb;
    for (int p = 0; p < s; ++p) fpos[nd.S[p]] = p;
    for (int q = 0; q < t; ++q) fpos[nd.R[q]] = s + q;
    Fm.assign(static_cast<size_t>(m) * m, 0.0);
    // original entries of the S columns: F(row u, col v) for u in S or R (pose rows of earlier
    // supernodes were eliminated there); BSR block (v, u) column-major = block (u, v) row-major
    for (int p = 0; p < s; ++p) {
      const int v = nd.S[p];
      for (int k = rowptr[v]; k < rowptr[v + 1]; ++k) {
        const int q = fpos[col[k]];
        if (q < 0) continue;
        const double* src = &blocks_colmajor[static_cast<size_t>(k) * bb];
        for (int i = 0; i < b; ++i)
          for (int j = 0; j < b; ++j) Fm[static_cast<size_t>(q * b + i) * m + p * b + j] += src[i * b + j];
      }
      for (int i = 0; i < b; ++i) Fm[static_cast<size_t>(p * b + i) * m + p * b + i] += shift;
    }
    for (int c : nd.children) {  // extend-add (children in order: deterministic)
      const SnNode& ch = nodes[c];
      const int tc = static_cast<int>(ch.R.size()), tcb = tc * b;
      const std::vector<double>& U = upd[c];
      for (int i = 0; i < tc; ++i)
        for (int ii = 0; ii < b; ++ii) {
          const double* ur = &U[static_cast<size_t>(i * b + ii) * tcb];
          double* fr = &Fm[static_cast<size_t>(ch.to_parent[i] * b + ii) * m];
          for (int j = 0; j < tc; ++j) {
            const int fc = ch.to_parent[j] * b;
            for (int jj = 0; jj < b; ++jj) fr[fc + jj] += ur[j * b + jj];
          }
        }
      std::vector<double>().swap(upd[c]);
    }
    for (int v : nd.S) fpos[v] = -1;
    for (int v : nd.R) fpos[v] = -1;
    // F_SS = L_SS L_SS^T; L_RS = F_RS L_SS^-T; U = F_RR - L_RS L_RS^T
    if (!potrf(Fm.data(), sb, m)) {
      err = "exact preconditioner: Q + 0.1 I is not positive definite";
      return -1;
    }
    double* LRS = Fm.data() + static_cast<size_t>(sb) * m;
    trsm_right_lt(LRS, tb, sb, m, Fm.data(), m);
    if (nd.parent >= 0 && tb > 0) {
      std::vector<double>& U = upd[x];
      U.assign(static_cast<size_t>(tb) * tb, 0.0);
      for (int i = 0; i < tb; ++i)
        std::memcpy(&U[static_cast<size_t>(i) * tb], LRS + static_cast<size_t>(i) * m + sb, sizeof(double) * tb);
      syrk_sub(U.data(), tb, LRS, tb, sb, m);
    }
    // panel = [L_SS^-1 ; L_RS L_SS^-1] in tiles
    Linv.assign(static_cast<size_t>(sb) * sb, 0.0);
    if (sb > 0) trtri_lower(Fm.data(), sb, m, Linv.data());
    M.assign(static_cast<size_t>(tb) * sb, 0.0);
    if (sb > 0 && tb > 0) trmm_right_lower(LRS, tb, sb, m, Linv.data(), M.data());
    const int S_pad = sn_pad(sb), R_pad = sn_pad(tb), ns = S_pad / kSnTile, nr = R_pad / kSnTile;
    nd.panel.assign(static_cast<size_t>(sn_panel_tiles(sb, tb)) * kSnTile * kSnTile, 0.0);
    for (int I = 0; I < ns + nr; ++I)
      for (int J = 0; J < ns && (I >= ns || J <= I); ++J) {
        double* tile = &nd.panel[static_cast<size_t>(sn_tile_index(ns, I, J)) * kSnTile * kSnTile];
        for (int u = 0; u < kSnTile; ++u)
          for (int v = 0; v < kSnTile; ++v) {
            const int c = J * kSnTile + v;
            if (c >= sb) continue;
            double val = 0.0;
            if (I < ns) {
              const int rr = I * kSnTile + u;
              if (rr < sb && c <= rr) val = Linv[static_cast<size_t>(rr) * sb + c];
            } else {
              const int rr = (I - ns) * kSnTile + u;
              if (rr < tb) val = M[static_cast<size_t>(rr) * sb + c];
            }
            tile[u * kSnTile + v] = val;
          }
      }
  }
  return 0;
}

// Host solve P x = rhs with the panels (the GPU sweeps' arithmetic, one right-hand side): the host
// chordal initialisation's direct solver.  rhs: n b values in pose order, overwritten with x.
void supernodal_solve(const SupernodalFactor& F, std::vector<double>& rhs) {
  const int b = F.b, nn = static_cast<int>(F.nodes.size());
  constexpr int T = kSnTile;
  int maxd = 0;
  for (const auto& nd : F.nodes) maxd = std::max(maxd, nd.depth);
  std::vector<double> y(rhs.size(), 0.0), x(rhs.size(), 0.0), f;
  std::vector<std::vector<double>> U(nn);
  for (int dep = maxd; dep >= 0; --dep)
    for (int id = 0; id < nn; ++id) {
      const SnNode& nd = F.nodes[id];
      if (nd.depth != dep) continue;
      const int s = static_cast<int>(nd.S.size()), t = static_cast<int>(nd.R.size()), sb = s * b, tb = t * b;
      const int Sp = sn_pad(sb), Rp = sn_pad(tb), ns = Sp / T, nr = Rp / T;
      f.assign(static_cast<size_t>(Sp + Rp), 0.0);
      for (int p = 0; p < s; ++p)
        for (int k = 0; k < b; ++k) f[p * b + k] = rhs[static_cast<size_t>(nd.S[p]) * b + k];
      for (int c : nd.children) {
        const SnNode& ch = F.nodes[c];
        for (size_t i = 0; i < ch.R.size(); ++i) {
          const int pos = ch.to_parent[i], row0 = pos < s ? pos * b : Sp + (pos - s) * b;
          for (int k = 0; k < b; ++k) f[row0 + k] += U[c][i * b + k];
        }
        std::vector<double>().swap(U[c]);
      }
      U[id].assign(static_cast<size_t>(tb), 0.0);
      for (int I = 0; I < ns + nr; ++I)
        for (int u = 0; u < T; ++u) {
          const int row = I * T + u;
          double out = 0.0;
          for (int J = 0; J < ns && (I >= ns || J <= I); ++J) {
            const double* tile = &nd.panel[static_cast<size_t>(sn_tile_index(ns, I, J)) * T * T + u * T];
            out += dot(tile, &f[J * T], T);
          }
          if (row < sb) y[static_cast<size_t>(nd.S[row / b]) * b + row % b] = out;
          else if (row >= Sp && row - Sp < tb) U[id][row - Sp] = f[row] - out;
        }
    }
  std::vector<double> g;
  for (int dep = 0; dep <= maxd; ++dep)
    for (int id = 0; id < nn; ++id) {
      const SnNode& nd = F.nodes[id];
      if (nd.depth != dep) continue;
      const int s = static_cast<int>(nd.S.size()), t = static_cast<int>(nd.R.size()), sb = s * b, tb = t * b;
      const int Sp = sn_pad(sb), Rp = sn_pad(tb), ns = Sp / T, nr = Rp / T;
      g.assign(static_cast<size_t>(Sp + Rp), 0.0);
      for (int row = 0; row < sb; ++row) g[row] = y[static_cast<size_t>(nd.S[row / b]) * b + row % b];
      for (int rr = 0; rr < tb; ++rr) g[Sp + rr] = -x[static_cast<size_t>(nd.R[rr / b]) * b + rr % b];
      for (int c = 0; c < sb; ++c) {
        const int J = c / T, v = c % T;
        double out = 0.0;
        for (int I = J; I < ns + nr; ++I) {
          const double* tile = &nd.panel[static_cast<size_t>(sn_tile_index(ns, I, J)) * T * T + v];
          for (int u = 0; u < T; ++u) out += tile[u * T] * g[I * T + u];
        }
        x[static_cast<size_t>(nd.S[c / b]) * b + c % b] = out;
      }
    }
  rhs.swap(x);
}

}  // namespace dpgo

// Host block Cholesky of P = Q + shift I for the exact preconditioner (QuadraticProblem::setQ,
// src/QuadraticProblem.cpp:37-41 factorises Q + 0.1 I with CHOLMOD; PreConditioner :75-87 applies
// it).  Built once per Q, on the host like the reference's factorisation; the per-iteration
// triangular solves run on the GPU (kernels.hip, k_trsv_level).
//
// Granularity is the pose block (b x b): the pose graph is ordered by recursive nested dissection
// (BFS level-structure separators), the block elimination tree gives the column patterns, and a
// left-looking block factorisation fills them.  The result is exact up to rounding, like CHOLMOD's
// (which orders and factorises differently, so bits differ but P^-1 v agrees to cond(P) * eps).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <queue>
#include <string>
#include <vector>

#include "chol_internal.h"

namespace dpgo {

namespace {

// BFS from s over the vertices with mark == tag; returns levels (vertex lists) and the last vertex.
int bfs_levels(const std::vector<std::vector<int>>& adj, int s, const std::vector<int>& mark, int tag,
               std::vector<int>& level, std::vector<std::vector<int>>& levels) {
  levels.clear();
  std::vector<int> cur{s}, nxt;
  level[s] = 0;
  int last = s;
  while (!cur.empty()) {
    levels.push_back(cur);
    nxt.clear();
    for (int v : cur)
      for (int u : adj[v])
        if (mark[u] == tag && level[u] < 0) {
          level[u] = static_cast<int>(levels.size());
          nxt.push_back(u);
        }
    if (!nxt.empty()) last = nxt.back();
    cur.swap(nxt);
  }
  return last;
}

// Nested dissection: order[] receives vertices, separators after both halves (eliminated last).
void nested_dissection(const std::vector<std::vector<int>>& adj, std::vector<int> verts, std::vector<int>& mark,
                       int& next_tag, std::vector<int>& order, std::vector<int>& level) {
  const size_t kLeaf = 64;
  if (verts.size() <= kLeaf) {
    // small part: minimum-degree-ish (ascending degree within the part) is plenty here
    std::sort(verts.begin(), verts.end(), [&](int a, int b) {
      return adj[a].size() != adj[b].size() ? adj[a].size() < adj[b].size() : a < b;
    });
    for (int v : verts) order.push_back(v);
    return;
  }
  const int tag = next_tag++;
  for (int v : verts) {
    mark[v] = tag;
    level[v] = -1;
  }
  // connected components first
  std::vector<std::vector<int>> comps;
  for (int v : verts) {
    if (level[v] >= 0) continue;
    std::vector<std::vector<int>> lv;
    bfs_levels(adj, v, mark, tag, level, lv);
    std::vector<int> comp;
    for (auto& l : lv) comp.insert(comp.end(), l.begin(), l.end());
    comps.push_back(std::move(comp));
  }
  if (comps.size() > 1) {
    for (auto& c : comps) nested_dissection(adj, std::move(c), mark, next_tag, order, level);
    return;
  }
  // pseudo-peripheral start: two sweeps
  for (int v : verts) level[v] = -1;
  std::vector<std::vector<int>> lv;
  int far = bfs_levels(adj, verts[0], mark, tag, level, lv);
  for (int v : verts) level[v] = -1;
  bfs_levels(adj, far, mark, tag, level, lv);
  if (lv.size() < 3) {  // no useful separator (dense-ish part): order as is
    for (int v : verts) order.push_back(v);
    return;
  }
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
  nested_dissection(adj, std::move(A), mark, next_tag, order, level);
  nested_dissection(adj, std::move(B), mark, next_tag, order, level);
  for (int v : S) order.push_back(v);
}

}  // namespace

int block_cholesky(int n, int b, const std::vector<int>& rowptr, const std::vector<int>& col,
                   const std::vector<double>& blocks_colmajor, double shift, size_t max_blocks, BlockCholesky& L,
                   std::string& err) {
  const int bb = b * b;
  // ---- ordering on the pose graph
  std::vector<std::vector<int>> adj(n);
  for (int j = 0; j < n; ++j)
    for (int k = rowptr[j]; k < rowptr[j + 1]; ++k)
      if (col[k] != j) adj[j].push_back(col[k]);
  for (auto& a : adj) {
    std::sort(a.begin(), a.end());
    a.erase(std::unique(a.begin(), a.end()), a.end());
  }
  std::vector<int> all(n), mark(n, -1), level(n, -1), order;
  std::iota(all.begin(), all.end(), 0);
  int tag = 0;
  order.reserve(n);
  nested_dissection(adj, all, mark, tag, order, level);
  L.n = n;
  L.b = b;
  L.perm = order;  // perm[new] = old
  L.iperm.assign(n, 0);
  for (int i = 0; i < n; ++i) L.iperm[order[i]] = i;
  // ---- symbolic: elimination tree + column patterns (new indices), adj+ (later neighbours)
  std::vector<std::vector<int>> pat(n);
  std::vector<int> parent(n, -1);
  std::vector<std::vector<int>> children(n);
  size_t total = 0;
  std::vector<int> flag(n, -1);
  for (int j = 0; j < n; ++j) {
    std::vector<int>& P = pat[j];
    flag[j] = j;
    P.push_back(j);
    for (int u : adj[order[j]]) {
      const int i = L.iperm[u];
      if (i > j && flag[i] != j) {
        flag[i] = j;
        P.push_back(i);
      }
    }
    for (int c : children[j])
      for (int i : pat[c])
        if (i > j && flag[i] != j) {
          flag[i] = j;
          P.push_back(i);
        }
    std::sort(P.begin() + 1, P.end());
    if (P.size() > 1) {
      parent[j] = P[1];
      children[P[1]].push_back(j);
    }
    total += P.size();
    if (total > max_blocks) {
      err = "exact preconditioner: the Cholesky factor of Q + 0.1 I would exceed " + std::to_string(max_blocks) +
            " pose blocks (use DPGO_PRECON_BLOCK_JACOBI for this size)";
      return -1;
    }
  }
  L.colptr.assign(n + 1, 0);
  for (int j = 0; j < n; ++j) L.colptr[j + 1] = L.colptr[j] + static_cast<int>(pat[j].size());
  L.rowidx.resize(total);
  for (int j = 0; j < n; ++j) std::copy(pat[j].begin(), pat[j].end(), L.rowidx.begin() + L.colptr[j]);
  std::vector<std::vector<int>>().swap(pat);
  std::vector<std::vector<int>>().swap(children);
  // ---- numeric, left-looking: column j = P(:, j) - sum_{k: L(j,k) != 0} L(:, k) L(j, k)^T
  L.blocks.assign(total * bb, 0.0);
  // row lists: for each row j, the columns k < j with L(j,k) != 0 and the block offset
  std::vector<std::vector<std::pair<int, long>>> rows(n);
  for (int k = 0; k < n; ++k)
    for (int p = L.colptr[k] + 1; p < L.colptr[k + 1]; ++p) rows[L.rowidx[p]].push_back({k, static_cast<long>(p)});
  std::vector<long> where(n, -1);
  for (int j = 0; j < n; ++j) {
    for (int p = L.colptr[j]; p < L.colptr[j + 1]; ++p) where[L.rowidx[p]] = p;
    // scatter P(:, j) (column j in new order = column order[j] of P): block (i, j) row-major
    const int oj = order[j];
    for (int k = rowptr[oj]; k < rowptr[oj + 1]; ++k) {
      const int i = L.iperm[col[k]];
      if (i < j) continue;
      // BSR block (oj, col[k]) column-major = block (col[k], oj) row-major  (Q symmetric)
      double* dst = &L.blocks[where[i] * bb];
      const double* src = &blocks_colmajor[static_cast<size_t>(k) * bb];
      for (int x = 0; x < bb; ++x) dst[x] += src[x];
    }
    for (int u = 0; u < b; ++u) L.blocks[where[j] * bb + u * b + u] += shift;
    // updates from columns k with L(j,k) != 0
    for (const auto& [k, pjk] : rows[j]) {
      const double* Ljk = &L.blocks[pjk * bb];
      for (int p = static_cast<int>(pjk); p < L.colptr[k + 1]; ++p) {  // rows i >= j of column k
        const double* Lik = &L.blocks[static_cast<size_t>(p) * bb];
        double* dst = &L.blocks[where[L.rowidx[p]] * bb];
        for (int u = 0; u < b; ++u)
          for (int v = 0; v < b; ++v) {
            double s = 0.0;
            for (int w = 0; w < b; ++w) s += Lik[u * b + w] * Ljk[v * b + w];
            dst[u * b + v] -= s;
          }
      }
    }
    // dense Cholesky of the diagonal block, then L(i,j) = A(i,j) L(j,j)^-T
    double* D = &L.blocks[where[j] * bb];
    for (int c = 0; c < b; ++c) {
      double d = D[c * b + c];
      for (int w = 0; w < c; ++w) d -= D[c * b + w] * D[c * b + w];
      if (!(d > 0.0)) {
        err = "exact preconditioner: Q + 0.1 I is not positive definite";
        return -1;
      }
      d = std::sqrt(d);
      D[c * b + c] = d;
      for (int u = c + 1; u < b; ++u) {
        double s = D[u * b + c];
        for (int w = 0; w < c; ++w) s -= D[u * b + w] * D[c * b + w];
        D[u * b + c] = s / d;
      }
      for (int u = 0; u < c; ++u) D[u * b + c] = 0.0;  // keep the block lower triangular
    }
    for (int p = L.colptr[j] + 1; p < L.colptr[j + 1]; ++p) {
      double* A = &L.blocks[static_cast<size_t>(p) * bb];
      for (int u = 0; u < b; ++u)  // row u of A: solve x L(j,j)^T = a  (forward over columns)
        for (int c = 0; c < b; ++c) {
          double s = A[u * b + c];
          for (int w = 0; w < c; ++w) s -= A[u * b + w] * D[c * b + w];
          A[u * b + c] = s / D[c * b + c];
        }
    }
    for (int p = L.colptr[j]; p < L.colptr[j + 1]; ++p) where[L.rowidx[p]] = -1;
  }
  return 0;
}

}  // namespace dpgo

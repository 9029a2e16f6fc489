// Host supernodal Cholesky for the exact preconditioner (chol.cpp) -- internal, not ABI.
#pragma once
#include <string>
#include <vector>

namespace dpgo {

// Panels are stored in square tiles of kSnTile x kSnTile scalars (row-major inside a tile).
constexpr int kSnTile = 64;

inline int sn_pad(int scalars) { return (scalars + kSnTile - 1) / kSnTile * kSnTile; }

// One supernode of the nested-dissection tree of an agent's pose graph (a separator, or a leaf part
// eliminated as one dense block).  Its columns are the poses S (in elimination order); R lists the
// poses of its ancestors its factor column block reaches (the row structure below S).  In the factor
// P = L L^T, the block column of S is [L_SS; L_RS].  The GPU solves use, per supernode, the panel
//   Panel = [L_SS^-1 ; L_RS L_SS^-1]      ((s + t) b x s b scalars, s = |S|, t = |R|)
// so both triangular sweeps are dense products with no dependency inside a supernode:
//   forward  L y = v:    f = [v_S + children's updates ; children's updates on R]
//                        y_S = L_SS^-1 f_S,   u = f_R - (L_RS L_SS^-1) f_S   (passed to the parent)
//   backward L^T x = y:  x_S = L_SS^-T y_S - (L_RS L_SS^-1)^T x_R
// Scalar rows: S part rows [0, s b) padded to S_pad = sn_pad(s b), then R part rows [S_pad, S_pad + t b)
// padded to R_pad; columns [0, S_pad).  Tiles: row tile I < S_pad / kSnTile holds column tiles 0..I
// (the lower-triangular L_SS^-1; tiles above the diagonal are not stored), every other row tile holds
// all S_pad / kSnTile column tiles.  Padding is zero.
struct SnNode {
  std::vector<int> S, R;   // agent-local pose ids
  int parent = -1;
  std::vector<int> children;
  int depth = 0;           // distance from the root of the agent's tree
  std::vector<int> to_parent;  // R[i] -> its position in the parent's frontal order (S_parent, then R_parent)
  std::vector<double> panel;
};

inline long sn_panel_tiles(int s_scalars, int t_scalars) {
  const long ns = sn_pad(s_scalars) / kSnTile, nr = sn_pad(t_scalars) / kSnTile;
  return ns * (ns + 1) / 2 + nr * ns;
}
inline long sn_tile_index(int ns_tiles, int I, int J) {
  return I < ns_tiles ? static_cast<long>(I) * (I + 1) / 2 + J
                      : static_cast<long>(ns_tiles) * (ns_tiles + 1) / 2 + static_cast<long>(I - ns_tiles) * ns_tiles + J;
}

struct SupernodalFactor {
  int n = 0, b = 0;
  std::vector<SnNode> nodes;  // postorder: every child before its parent; the root last
  long panel_doubles = 0;
};

// The symbolic half of supernodal_cholesky: the nested-dissection tree, every node's S and R (elimination
// order), the extend-add maps (to_parent) and panel_doubles; no values (the pattern of Q only; blocks unused).
// Returns 0, or -1 with err set (the panels would exceed max_doubles).  The device factorisation
// (kernels.hip k_sn_factor) runs its numeric half on this structure.
int supernodal_symbolic(int n, int b, const std::vector<int>& rowptr, const std::vector<int>& col, long max_doubles,
                        SupernodalFactor& F, std::string& err);

// Factorise P = Q + shift I, Q given as symmetric block-sparse rows (block (j, col) column-major), over
// the nested-dissection supernodes of its block graph (multifrontal, dense frontal matrices).  Returns 0,
// or -1 with err set (not positive definite, or the panels would exceed max_doubles).
int supernodal_cholesky(int n, int b, const std::vector<int>& rowptr, const std::vector<int>& col,
                        const std::vector<double>& blocks_colmajor, double shift, long max_doubles,
                        SupernodalFactor& F, std::string& err);

// Host solve (L L^T) x = rhs in place with the panels (one right-hand side, n b values in pose order).
void supernodal_solve(const SupernodalFactor& F, std::vector<double>& rhs);

}  // namespace dpgo

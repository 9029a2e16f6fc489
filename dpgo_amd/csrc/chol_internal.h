// Host block Cholesky for the exact preconditioner (chol.cpp) -- internal, not ABI.
#pragma once
#include <string>
#include <vector>

namespace dpgo {

// P = L L^T over pose blocks in elimination order: column j (new index) lists its rows (new
// indices, the first is j itself, the rest ascending) with b x b blocks L(i, j) row-major; the
// diagonal blocks are lower triangular.  perm[new] = old pose index, iperm[old] = new.
struct BlockCholesky {
  int n = 0, b = 0;
  std::vector<int> perm, iperm;
  std::vector<int> colptr, rowidx;
  std::vector<double> blocks;
};

// Factorise P = Q + shift I, Q given as symmetric block-sparse rows (block (j, col) column-major).
// Returns 0, or -1 with err set (not positive definite, or more than max_blocks factor blocks).
int block_cholesky(int n, int b, const std::vector<int>& rowptr, const std::vector<int>& col,
                   const std::vector<double>& blocks_colmajor, double shift, size_t max_blocks, BlockCholesky& L,
                   std::string& err);

}  // namespace dpgo

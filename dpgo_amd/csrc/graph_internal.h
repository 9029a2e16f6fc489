// Internal (non-ABI) pose-graph representation shared by graph.cpp and rbcd.cpp.
#pragma once
#include <string>
#include <vector>

#include "../../include/dpgo_rbcd.h"
#include "problem_internal.h"

struct dpgo_graph_s {
  int d = 0, n = 0, duplicates = 0;
  std::vector<int> r1, r2, p1, p2;
  std::vector<double> R, t, kappa, tau;  // R row-major d*d per edge
  std::vector<int> coords;               // grid graphs: (x, y, z) per pose
  dpgo::HostBSR q_cache;
  bool q_cache_valid = false;
};

namespace dpgo {

// Two-pass BSR assembly: touch() the structure, freeze(), then accumulate blocks with add().
struct BsrBuilder {
  int n = 0, b = 0;
  std::vector<std::vector<int>> cols;
  HostBSR out;
  BsrBuilder(int n_, int b_) : n(n_), b(b_), cols(n_) {
    for (int j = 0; j < n_; ++j) cols[j].push_back(j);  // every pose keeps a diagonal block
  }
  void touch(int i, int j) { cols[i].push_back(j); }
  void freeze();
  double* block(int i, int j);  // column-major b x b block (i, j)
  void add(int i, int j, const double* blk);
};

void edge_blocks(int d, const double* R, const double* t, double kappa, double tau, double w, double* Wii,
                 double* Wjj, double* Wij, double* Wji);

// chordalInitialization (src/DPGO_utils.cpp:377-424), init.cpp: T_out d x (d+1) n column-major
int chordal_initialization(int d, int n, int m, const int* p1, const int* p2, const double* R, const double* t,
                           const double* kappa, const double* tau, double* T_out, std::string& err);
// same minimiser, both linear solves by Jacobi-PCG on the GPU (|r| <= rtol |b| per right-hand side)
int chordal_initialization_gpu(int d, int n, int m, const int* p1, const int* p2, const double* R, const double* t,
                               const double* kappa, const double* tau, double* T_out, double rtol, int max_iters,
                               int* iters, double* relres, std::string& err);
// PGOAgent::localInitialization (chordal per agent on its private graph, anchored at the agent's BFS
// centre) + initializeInGlobalFrame (breadth-first L2 alignment over shared loop closures)
// projectToRotationGroup of a d x d row-major matrix (init.cpp)
void project_to_rotation(int d, const double* M, double* out);

int distributed_initialization(int d, int n, int m, const int* p1, const int* p2, const double* R, const double* t,
                               const double* kappa, const double* tau, const int* agent_of, int num_agents, bool gpu,
                               double rtol, int max_iters, double* T_out, int* iters, double* relres,
                               std::string& err);

}  // namespace dpgo

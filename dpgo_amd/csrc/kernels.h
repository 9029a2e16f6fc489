// Launch-side view of the DPGO HIP kernels (shared by kernels.hip and the C-ABI layer).
#pragma once
#include <hip/hip_runtime.h>

#include "dpgo_device.h"

namespace dpgo {

constexpr int kPartialStride = 4;  // doubles of partial sums per tile

enum SpmmMode { MODE_XQ = 0, MODE_XQ_G = 1, MODE_EVAL = 2, MODE_HESS = 3 };
enum FlagKind { FLAG_NONE = 0, FLAG_RUN = 1, FLAG_TCG = 2, FLAG_TCG_MODE = 3 };
enum PreconMode { PRECON_EXACT = 0, PRECON_BLOCK_JACOBI = 1, PRECON_NONE = 2 };
enum TcgStatus { TCG_NEGCURVTURE = 0, TCG_EXCREGION = 1, TCG_LCON = 2, TCG_SCON = 3, TCG_MAXITER = 4 };
enum FinalizeOp {
  OP_EVAL_INIT = 0,
  OP_EVAL = 1,
  OP_TCG_INIT = 2,
  OP_TCG_STEP = 3,
  OP_TCG_CHECK = 4,
  OP_RHO = 5,
  OP_REL_CHANGE = 6,
  OP_SUM = 7
};

// Tile set + per-agent state for one launch.
struct LaunchCtx {
  const int* tile_agent;  // [num_tiles]
  const int* tile_start;  // [num_tiles] first (global, concatenated) pose of the tile
  const int* tile_count;  // [num_tiles] poses in the tile (<= 64)
  int num_tiles;
  int flag_kind;          // FlagKind: which per-agent flag gates the tile
  AgentState* state;      // [num_agents] (may be null with FLAG_NONE)
  double* partials;       // [num_tiles * kPartialStride]
  hipStream_t stream;
};

// Block-sparse (BSR) symmetric Q over the concatenated poses of all agents in the batch.
struct QView {
  const int* rowptr;      // [n + 1]
  const int* col;         // [nnzb] global pose index
  const double* blocks;   // [nnzb * b * b], block (j, col) column-major
};

struct OptScalars {
  double tol, Delta0, Delta_max, theta, kappa;
  int min_inner, max_iter, single_run, pad;
};

struct FinalizeArgs {
  int op;
  int nq_a, nq_b;
  const int* agent_tile_off;    // [num_agents + 1]
  const int* agent_num_poses;   // [num_agents]
  const int* agent_enabled;     // optional [num_agents]
  const double* pa;
  const double* pb;
  AgentState* state;
  double* out_sums;             // OP_SUM: [num_agents * 4]
  OptScalars opt;
  // zero-copy status publication to host-mapped memory: pub[agent] = (tag << 1) | flag
  int* pub;                     // nullptr = none
  int pub_tag;
  int pub_kind;                 // 1: tcg_active, 2: run_active
};

// shared-edge records for G assembly, grouped by G slot (CSR)
struct GEdges {
  const int* slot_off;   // [nslots + 1]
  const int* src;        // neighbour pose: >= 0 index into Xa, < 0 -> (-1 - src) into Xb
  const int* outgoing;   // 1: this agent owns p1 (edge leaves the agent)
  const double* R;       // [d*d] row-major per edge
  const double* t;       // [d]
  const double* kappa;
  const double* tau;
  const double* w;
};

// Runtime-selectable kernel variants (A/B tuning in one process; see tools/spmm_ab.py).
enum TuneKey { TUNE_SPMM_VARIANT = 0, TUNE_COUNT = 4 };
extern int g_tuning[TUNE_COUNT];

bool supported_rb(int r, int b);
hipError_t launch_gather_poses(int count, int rb, const int* idx, const double* A, const double* Bsrc, double* dst,
                               hipStream_t stream);
hipError_t launch_assemble_G(int r, int b, const GEdges& e, int nslots, const double* Xa, const double* Xb,
                             double* gblk, hipStream_t stream);
hipError_t launch_spmm(int r, int b, int mode, const LaunchCtx& c, const QView& q, const double* in,
                       const int* gidx, const double* gblk, const double* X, const double* S_in,
                       double* out, double* S_out);
hipError_t launch_tcg_init(int r, int b, const LaunchCtx& c, const double* X, const double* Minv, int pmode,
                           const double* g, double* delta);
hipError_t launch_tcg_update(int r, int b, const LaunchCtx& c, const double* X, const double* Minv, int pmode,
                             const double* delta, const double* Hdelta, double* eta, double* Heta,
                             const double* r_in, double* rv, double* z, int first);
hipError_t launch_tcg_dir(int r, int b, const LaunchCtx& c, const double* z, double* delta);
hipError_t launch_retract(int r, int b, const LaunchCtx& c, const double* X, const double* V, double scale,
                          double* out, const double* g, const double* HV);
hipError_t launch_tangent(int r, int b, const LaunchCtx& c, const double* X, const double* V, double* out);
hipError_t launch_precond(int r, int b, const LaunchCtx& c, const double* X, const double* Minv, int pmode,
                          const double* V, double* out);
hipError_t launch_polar_comb(int r, int b, const LaunchCtx& c, const double* A, const double* Bv,
                             const double* ca, const double* cb, double* out, const double* Cv = nullptr,
                             double sa = 1.0, double sb = 0.0, double* out2 = nullptr);
hipError_t launch_select(int r, int b, const LaunchCtx& c, const double* A, const double* Bv, const int* use_a,
                         const double* ref, double* out);
hipError_t launch_accept(int r, int b, const LaunchCtx& c, const double* x2, const double* g2, const double* S2,
                         double* x1, double* g, double* S);
hipError_t launch_finalize(const FinalizeArgs& f, int num_agents, hipStream_t stream);
hipError_t launch_bj_inverse(int b, int n, const QView& q, double shift, double* Minv, hipStream_t stream);

}  // namespace dpgo

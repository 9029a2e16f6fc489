// Launch-side view of the DPGO HIP kernels (shared by kernels.hip and the C-ABI layer).
#pragma once
#include <hip/hip_runtime.h>

#include "dpgo_device.h"

namespace dpgo {

constexpr int kPartialStride = 16;  // doubles of partial sums per tile
constexpr int kDdLo = 8;  // a double-double partial keeps its low part this many slots after its high part
constexpr int kMaxTot = 8;         // quantities one finalize reduces (pa + pb, and pc at the last slot)

// X.Q SpMM epilogues: XQ (V Q), XQ_G (X Q + G), EVAL (g = P_X(XQ+G), S, f / |g|^2 partials),
// HESS (Riemannian Hessian), F (f partial only), EVAL_TCG (EVAL + tCG start: delta = -P_X(g Minv),
// partial <z, g>)
// CERT: V (Q - Lambda(X)) = VQ - [V_Y S | 0] (the certificate matrix, no projection)
// HESS_M / HESS_QF_M (the merged tCG iteration): HESS / HESS_QF plus the partials the stopping test and
// beta need as polynomials in alpha (|r|^2, <r,Hd>, |Hd|^2, <z,r>, 2<z,Hd>, <Minv Hd,Hd>, see k_spmm)
enum SpmmMode { MODE_XQ = 0, MODE_XQ_G = 1, MODE_EVAL = 2, MODE_HESS = 3, MODE_F = 4, MODE_EVAL_TCG = 5, MODE_CERT = 6,
                MODE_QF = 7, MODE_HESS_QF = 8, MODE_HESS_M = 9, MODE_HESS_QF_M = 10 };
constexpr int kSpmmModes = 11;
__host__ __device__ constexpr bool mode_merged(int m) { return m == MODE_HESS_M || m == MODE_HESS_QF_M; }
__host__ __device__ constexpr bool mode_hess(int m) {
  return m == MODE_HESS || m == MODE_HESS_QF || m == MODE_HESS_M || m == MODE_HESS_QF_M;
}
__host__ __device__ constexpr bool mode_snap(int m) { return m == MODE_HESS_QF || m == MODE_HESS_QF_M; }
// Precision of the merged tCG partials (pa slots of MODE_HESS_M / MODE_HESS_QF_M, FinalizeArgs::dd_mask): bit s set
// = slot s is double-double.  kMergedDdSlotsV1 is the round-3 epilogue's (every quantity but d_Hd).  The v2
// epilogue (edge variant bit 6) keeps double-double where a sum cancels across poses and feeds beta: |r_0|^2
// and <z_0, r_0> (slots 1, 4: first iteration) always, the others as DPGO_MERGED_DD_SLOTS says -- <r,Hd> (2),
// |Hd|^2 (3), 2<z,Hd> (5), <Minv Hd,Hd> (6).  The default is the one test_rtr_trace_extended_precision and
// tools/trace_precision.py chose.
#ifndef DPGO_MERGED_DD_SLOTS
#define DPGO_MERGED_DD_SLOTS 0x20
#endif
constexpr int kMergedDdSlotsV1 = 0x7E;
constexpr int kMergedDdSlots = 0x12 | (DPGO_MERGED_DD_SLOTS & 0x6C);
// Per-agent tile gating: RUN skips agents out of the RTR Run, TCG those whose tCG stopped, TCG_MODE
// those with no tCG step pending, MOVED those whose single-Run candidate was accepted.
enum FlagKind { FLAG_NONE = 0, FLAG_RUN = 1, FLAG_TCG = 2, FLAG_TCG_MODE = 3, FLAG_MOVED = 4, FLAG_TCG_CG = 5,
                FLAG_RUN_IMPL = 6, FLAG_RUN_EXPL = 7,  // RUN_IMPL/EXPL: FLAG_RUN and eta (not) implicit
                FLAG_DECIDED = 8 };  // only agents whose single-Run outcome was decided in Run `round`
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
  OP_SUM = 7,
  OP_EVAL_TCG_INIT = 8,  // OP_EVAL_INIT then OP_TCG_INIT from one fused pass (f, |g|^2, <z,g>)
  OP_STATUS = 9,         // PGOAgent status: relativeChange = sqrt(|X - XPrev|^2 / n), readyToTerminate
  OP_TCG_STEP_CHECK = 10,  // merged tCG iteration: OP_TCG_STEP then OP_TCG_CHECK from one HESS_M pass
  OP_TCG_CHECK_M = 11      // OP_TCG_CHECK from a HESS_M pass whose step an earlier (MODE_QF) test decided
};

// Per-iteration trace (ROPTLIB ITERRESULT, src/QuadraticOptimizer.cpp:82-86): one record of
// kTraceWidth doubles per tCG step test, tCG stopping test and rho test, per agent.
constexpr int kTraceWidth = 16;
enum TraceField {
  TR_OP = 0,       // FinalizeOp that wrote the record (OP_TCG_STEP / OP_TCG_CHECK / OP_RHO)
  TR_J = 1,        // tCG iteration index (0-based) / RTR outer iteration
  TR_F1 = 2, TR_F2 = 3, TR_RHO = 4, TR_DELTA = 5,
  TR_ALPHA = 6, TR_BETA = 7, TR_TAU = 8, TR_DHD = 9, TR_NORM_R = 10, TR_ZR = 11,
  TR_STATUS = 12,  // tCG status when the record ends tCG / the Run, else -1
  TR_ACCEPTED = 13, TR_NGF = 14, TR_RUN = 15
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
  int round;              // FLAG_DECIDED: the RTR Run index (0-based)
  // edge-stream Q only (else null): per tile {first incidence, incidences, first first-visit record, records}, so a
  // launch issues the tile's stage loads right after the tile's scalar header instead of after a round trip
  // through its poses' incidence pointers
  const int4* tile_meta;
};

enum QFormat { QFMT_BSR = 0, QFMT_EDGES = 1 };

// Edge record: M = T Omega (b x b, T = [R t; 0 1], Omega = diag(w kappa I_d, w tau)) with rows
// padded to 4 doubles, so Q_{p1 p2} = -M and Q_{p2 p1} = -M^T are read straight from it.
__host__ __device__ constexpr int edge_rec_width(int d) { return 4 * (d + 1); }
// Packed symmetric diagonal block Q_jj (upper triangle, row-major): b (b + 1) / 2 doubles per pose.
__host__ __device__ constexpr int diag_width(int d) { return (d + 1) * (d + 2) / 2; }

// The symmetric Q over the concatenated poses of all agents in the batch, in one of two forms:
//  QFMT_BSR    block-sparse rows: any symmetric Q (QuadraticProblem::setQ).
//  QFMT_EDGES  the measurement stream Q = A Omega A^T is built from (src/DPGO_utils.cpp:214-286,
//              src/PGOAgent.cpp:720-781), never materialised as blocks: each edge's M = T Omega is
//              stored ONCE (both off-diagonal blocks are -M and -M^T) and every pose keeps its packed
//              diagonal block.  inc[k] = {2 * edge + (j == p1), other endpoint} lists the edges with
//              both endpoints in the batch (shared edges only feed the diagonal); edge ids follow
//              first-visit order so a tile's first-visit records are one contiguous range.
struct QView {
  const int* rowptr;      // BSR [n + 1]
  const int* col;         // BSR [nnzb] global pose index
  const double* blocks;   // BSR [nnzb * b * b], block (j, col) column-major
  const int* inc_ptr;     // EDGES [n + 1]
  const int2* inc;        // EDGES [nnz_inc]
  const double* rec;      // EDGES [m * edge_rec_width(d)]
  const double* diag;     // EDGES [n * diag_width(d)]
  const int* rec_first;   // EDGES [n + 1] first edge id first-visited by pose j (ids in visit order)
  // EDGES, second-visit staging (tile-indexed): sv_ids[sv_ptr[t] ..] = the ascending ids of the edges tile
  // t visits second; inc_sv = inc with tile-local record slots (second visits 0 .. ns-1 in that order,
  // first visit id -> ns + id - rec_first[tile's first pose]), the same ascending order per pose
  const int* sv_ptr;
  const int* sv_ids;
  const int2* inc_sv;
  int fmt;                // QFormat
  const int* tuning;      // host only: the handle's tuning keys (launch-time variant choice; kernels never read it)
};

struct OptScalars {
  double tol, Delta0, Delta_max, theta, kappa;
  double rel_tol, min_ratio;  // OP_STATUS: PGOAgentParameters relChangeTol, robustOptMinConvergenceRatio
  int min_inner, max_iter, single_run;
  int first_full;  // OP_TCG_STEP of a first step measured by MODE_HESS_QF (statistics only)
  int status_fold;  // OP_RHO of a single Run also sets the PGOAgent status of the agents it decides from
                    // k_retract's |x2 - ref|^2 / |x1 - ref|^2 partials (pa slots 2, 3)
};

struct FinalizeArgs {
  int op;
  int nq_a, nq_b;
  const int* agent_tile_off;    // [num_agents + 1]
  const int* agent_num_poses;   // [num_agents]
  const int* agent_enabled;     // optional [num_agents]
  const double* pa;
  const double* pb;
  const double* pc;             // third operand (nq_c quantities; the merged tCG's <eta, Hdelta> partials)
  int nq_c;
  AgentState* state;
  double* out_sums;             // OP_SUM: [num_agents * 4]
  OptScalars opt;
  // zero-copy status publication to host-mapped memory: pub[agent] = (tag << 1) | flag
  int* pub;                     // nullptr = none
  int pub_tag;
  int pub_kind;                 // 1: tcg_active, 2: run_active (+ bit 1: the Run's tCG took a CG step, bit 2:
                                // the agent never ran in this call)
  int agent_filter;             // 0: every agent; 1 / 2: only agents whose eta is / is not implicit
  int coherent;                 // read the partials with agent-scope loads (fused, SpmmArgs::fin_mode 2)
  const double* conv_ratio;     // OP_STATUS: per-agent converged loop-closure ratio (nullptr = 1)
  int dd_mask;                  // bit q: pa quantity q is double-double (low part at slot + kDdLo), reduced as such
  int rz_pc;                    // merged tCG: |r_j|^2 and <z_j, r_j> (quantities 1, 4) from the previous
                                // k_tcg_updir's double-double partials (pc slots 1, 2), not from pa
  double* trace;                // per-iteration records [agent][trace_cap][kTraceWidth] (nullptr = off)
  int trace_cap;
};

// SpMM modes that can run a fused finalize (SpmmArgs::fin_arrive); the others ignore it.
__host__ __device__ constexpr bool spmm_fusable(int mode) {
  return mode == MODE_EVAL || mode == MODE_EVAL_TCG || mode == MODE_F || mode == MODE_QF || mode == MODE_HESS ||
         mode == MODE_HESS_QF || mode == MODE_HESS_M || mode == MODE_HESS_QF_M;
}

// Operands of one SpMM launch (unused ones may be null).
struct SpmmArgs {
  const double* in;     // X (EVAL modes) or V
  const int* gidx;      // G slot per pose (-1 = none)
  const double* gblk;   // G blocks
  const double* X;      // iterate (EVAL / HESS)
  const double* S_in;   // cached sym(Y^T EG_Y) (HESS)
  double* out;          // result (gradient / HVP); may be null in EVAL
  double* S_out;        // S (EVAL)
  const double* Minv;   // block-Jacobi inverses (EVAL_TCG)
  double* delta;        // tCG direction (EVAL_TCG)
  int pmode;            // PreconMode (EVAL_TCG, HESS_M)
  const double* rvec;   // HESS_M: the tCG residual r_j (grad on the first iteration)
  int rz_own;           // HESS_M: also form the |r_j|^2 and <z_j, r_j> partials (else k_tcg_updir left them)
  // Fused finalize (null = none): the last block of each agent to arrive runs k_finalize's work for
  // that agent (fin), so no separate k_finalize launch follows the SpMM.  fin_arrive[agent] counts
  // arrivals and is reset to 0 by that last block.
  int* fin_arrive;
  int fin_mode;  // 1: device fences, 2: agent-scope partial stores and loads (see spmm_arrive)
  FinalizeArgs fin;
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
  const double* w;       // per entry weight, or null: 1
};

// The exact preconditioner's supernodal factor on the device (chol_internal.h: per supernode the panel
// [L_SS^-1 ; L_RS L_SS^-1] in kSnTileDev-square tiles), batch-global pose ids.  Frontal vectors F
// ((S_pad + R_pad) scalar rows x r) and update vectors U (t b rows x r) are work space.
constexpr int kSnTileDev = 64;
constexpr int kSnSmallNs = 2;  // k_sn_fwd_small: nodes of at most this many S column tiles
// One sweep item (supernode, tile) with everything its workgroup needs before its first data load: one 64-byte
// record instead of the item, then the node's agent, then the agent's flags, then the node's sizes and offsets --
// three dependent round trips ahead of the panel loads, which on the deep levels (tens of thousands of workgroups
// streaming 16-64 KB each) are most of a workgroup's life.
struct alignas(64) SnItem {
  int node, tile, agent, s, t, pad;
  long f_off, u_off, panel_off, cpanel_off, poses_off;  // cpanel_off -1: tiles only
};
static_assert(sizeof(SnItem) == 64, "one cache line per sweep item");

struct SnView {
  const double* panel;
  const long* panel_off;  // [nodes] first double of the node's panel
  const int* s;           // [nodes] poses in S
  const int* t;           // [nodes] poses in R
  const int* poses_off;   // [nodes] into poses: S then R
  const int* poses;
  const long* f_off;      // [nodes] into F
  const long* u_off;      // [nodes] into U
  const int* cpos_off;    // [nodes] into cpos: s + t + 1 pointers into contrib per node
  const int* cpos;
  const int2* contrib;    // per frontal position: (child node, index in the child's R), children in order
  double* F;
  double* U;
  // per-agent skip (the flag of the launch that consumes the sweep, k_precond_finish): a supernode's workgroups
  // exit when its agent's flag says so, so stopped agents cost no panel traffic
  const int* node_agent = nullptr;  // [nodes] batch agent of the node
  const AgentState* state = nullptr;
  int flag_kind = 0;
  // [agents] 1 where the agent's factorisation met a non-positive pivot: the reference's per-QuadraticProblem
  // fallback (src/QuadraticProblem.cpp:81-86, out = in unprojected) -- that agent's supernodes are skipped
  const int* ident = nullptr;
  // Narrow supernodes (at most kSnSmallNs S column tiles) are also kept compact: [L_SS^-1 ; L_RS L_SS^-1] as one
  // (s b + t b) x ld row-major matrix (ld = s b rounded up to 4) with none of the 64-row / 64-column tile padding
  // (deep nested-dissection levels: 2-2.4x padding).  cpanel_off[node] >= 0: the sweeps read it there instead of the
  // tiles (the same products in the same order, padding entries read as exact zeros); -1: tiles only.
  const double* cpanel = nullptr;
  const long* cpanel_off = nullptr;
  // per item of items_base (SnItem): k_sn_fwd, k_sn_fwd_small and k_sn_bwd read their item's record there (null:
  // from the arrays above)
  const SnItem* desc = nullptr;
  const int2* items_base = nullptr;
};

// The compact copy of the narrow supernodes' panels (SnView::cpanel) from their tiles: items (node, 64-row block of
// the compact matrix); launched after every factorisation
hipError_t launch_sn_compact(int b, const double* panel, const long* panel_off, const int* s, const int* t,
                             const long* cpanel_off, double* cpanel, const int2* items, int count, hipStream_t stream);
__host__ __device__ constexpr int sn_compact_ld(int sb) { return (sb + 3) / 4 * 4; }

// Numeric supernodal factorisation of P = Q + shift I on the device (k_sn_factor), over the symbolic structure the
// host built once (chol_internal.h supernodal_symbolic): one workgroup per supernode, one launch per tree level
// (deepest first).  Node g's dense frontal matrix (M x M row-major, M = S_pad + R_pad: the S rows padded to a
// kSnTileDev multiple, then the R rows) lives at F + f_off[g] in its level's buffer; its children's (one level
// deeper) in Fchild.  Assembly: the original entries of the S columns from the edge-stream Q (rec / diag, the
// current weights), then the children's update matrices (extend-add); then the blocked right-looking Cholesky
// over the S tile columns (leaving L_SS, L_RS and the update matrix U = F_RR - L_RS L_RS^T in place) and the
// panel [L_SS^-1 ; L_RS L_SS^-1] in the solve's tile layout.  Only the lower triangle of F is kept.
struct SnEntry {
  int q, p;    // frontal pose positions (row q >= column p; p in S)
  int s0, s1;  // edge sources src[s0 .. s1) (2 id + 1: block -M^T, 2 id: block -M); q == p: the diagonal block
};
struct SnFactorView {
  const int* nodes;       // this launch's node ids (one level)
  const int* s;           // [nodes] poses in S
  const int* t;           // [nodes] poses in R
  const long* f_off;      // [nodes] frontal offset in its level's buffer
  const long* panel_off;  // [nodes]
  const int* poses_off;   // [nodes] into poses: S then R (batch-global)
  const int* poses;
  const int* ch_off;      // [nodes + 1] into ch: children
  const int* ch;
  const int* tp_off;      // [nodes] into tp: the node's R entries' positions in its parent's frontal order
  const int* tp;
  const int* ent_off;     // [nodes + 1] into ent
  const SnEntry* ent;
  const int* src;
  const double* rec;      // edge-stream Q (current weights)
  const double* diag;
  double shift;
  double* F;              // this level's frontal buffer
  const double* Fchild;   // the level below
  double* panel;
  const int* node_agent;  // [nodes] batch agent of the node
  int* not_pd;            // [agents] set to 1 for the agent of a node that meets a non-positive pivot
};
// Loop closures one engine colour class reweights (PGOAgent::updateLoopClosuresWeights,
// src/PGOAgent.cpp:1181-1244): pose sources >= 0 index the engine's X buffer, < 0 -> (-1 - s) the
// received-pose buffer; weights go to the colour problem's edge and, for shared edges, its G entry.
// A shared loop closure reads the neighbour's pose from the agent's neighborPoseDict as the agent last received it
// (:1201-1235): `dict` holds that pose per entry (r b doubles), `dict_ok` whether the agent has received it yet (the
// reference skips an edge whose neighbour pose it does not have, weight unchanged); k_gnc_snapshot fills them when
// the agent is selected (the example delivers neighbour poses to the selected robot only,
// examples/MultiRobotExample.cpp:188-213).
struct GncEntries {
  int n;
  const int* prob_edge;
  const int* g_entry;  // -1: private loop closure
  const int* src1;
  const int* src2;
  const double* R;  // d*d row-major
  const double* t;
  const double* kappa;
  const double* tau;
  const int* agent;    // agent of the entry (index inside the colour problem)
  const int* nbr_end;  // shared entries: 1 if p2 is the neighbour's pose, 0 if p1; -1 private
  double* dict;        // per entry: the neighbour pose of the agent's dictionary
  int* dict_ok;
};
// RobustCost::weight (src/DPGO_robust.cpp:23-67) parameters; type = DPGO_ROBUST_*
struct RobustParams {
  int type;
  double mu, barc, huber, tls;
};

// Runtime-selectable kernel variants (A/B tuning in one process; see tools/spmm_ab.py).
enum TuneKey { TUNE_SPMM_VARIANT = 0, TUNE_EDGE_VARIANT = 1, TUNE_EPI_PREFETCH = 2, TUNE_FUSE_TCG = 3,
               TUNE_FIRST_STEP = 4,  // 0: predicted from the previous call, 1: always MODE_QF, 2: always MODE_HESS_QF
               TUNE_CLASSIC_TCG = 5,  // 1: five launches per tCG iteration (HESS, step test, update, check, dir)
                                      //    instead of the merged three (HESS_M, step + check, k_tcg_updir)
               TUNE_TCG_LOOKAHEAD = 7,  // merged single-Run tCG with the full first pass: 0 adaptive, 1 one
                                        // iteration queued ahead of a published status, 2 every iteration queued
               TUNE_MERGED_PREFETCH = 6,  // 1: HESS_M's r / Minv loaded before the edge loop (measured slower)
               TUNE_SV_STAGE = 8,  // 1: HESS passes stage the tile's second-visit records in LDS too (the
                                   //    tables are built when Q is set with this on; measured slower)
               TUNE_STATUS_PASS = 9,  // 1: the agent status by its own pass (k_sqdiff + OP_STATUS), not folded
               TUNE_SPLIT_STREAMS = 10,  // merged tCG queued at once: the batch's agents in two halves on two
                                         // streams (one half's VALU-bound HESS_M beside the other's HBM-bound
                                         // k_tcg_updir); 0 off, 1 on (default: 1M -0.7 %, the 125 k
                                         // share -4.6 % ms/step), 2 the halves out of phase (no gain),
                                         // 3 four agent groups on four streams, 4 one group per agent (<= 8)
               TUNE_DEVICE_CHOL = 12,  // exact preconditioner over an edge-stream Q: 1 numeric factorisation on the
                                       // device (k_sn_factor), 0 on the host (chol.cpp, panels uploaded)
               TUNE_SPMM_V2 = 11,  // > 0: the merged partials at kMergedDdSlots (edge variant bit 6) and the rotated
                                   //    accumulator (bit 7) in every mode (1), in none (2), in the merged modes (3);
                                   //    4: 3 + one edge-loop pipeline per pose in the merged modes (bit 8);
                                   //    5: rotated + one pipeline in every mode; 6 (default since round 5): 5 but the
                                   //    half passes (F, QF) plain; 0: the round-3 kernels
               TUNE_COUNT = 13 };
// dd_mask of the merged tCG partials for the kernel a handle with these tuning keys and Q format runs
inline int merged_dd_mask(int fmt, const int* tuning) {
  return fmt == QFMT_EDGES && tuning[TUNE_SPMM_V2] > 0 ? kMergedDdSlots : kMergedDdSlotsV1;
}
// variant of the edge-stream SpMM used unless TUNE_EDGE_VARIANT overrides it (bit 0: XCD-aware
// tile remap; v >> 1: minimum waves per SIMD the register allocation must allow, none/4/5/6)
constexpr int kEdgeDefaultVariant = 1;
extern int g_tuning[TUNE_COUNT];  // process defaults, copied into every handle at creation (dpgo_hip_set_tuning)

bool supported_rb(int r, int b);
hipError_t launch_gather_poses(int count, int rb, const int* idx, const double* A, const double* Bsrc, double* dst,
                               hipStream_t stream);
// dst pose idx[s] = src pose s, s < count
hipError_t launch_scatter_poses(int count, int rb, const int* idx, const double* src, double* dst, hipStream_t stream);
hipError_t launch_assemble_G(int r, int b, const GEdges& e, int nslots, const double* Xa, const double* Xb,
                             double* gblk, hipStream_t stream);
hipError_t launch_spmm(int r, int b, int mode, const LaunchCtx& c, const QView& q, const SpmmArgs& a);
inline hipError_t launch_spmm(int r, int b, int mode, const LaunchCtx& c, const QView& q, const double* in,
                              const int* gidx, const double* gblk, const double* X, const double* S_in,
                              double* out, double* S_out) {
  return launch_spmm(r, b, mode, c, q, SpmmArgs{in, gidx, gblk, X, S_in, out, S_out, nullptr, nullptr, PRECON_NONE});
}
hipError_t launch_tcg_init(int r, int b, const LaunchCtx& c, const double* X, const double* Minv, int pmode,
                           const double* g, double* delta);
hipError_t launch_tcg_update(int r, int b, const LaunchCtx& c, const double* X, const double* Minv, int pmode,
                             const double* delta, const double* Hdelta, double* eta,
                             const double* r_in, double* rv, double* z, int first,
                             const FinalizeArgs* fin = nullptr, int* arrive = nullptr);
// fin / arrive: the consumer-side finalize (OP_TCG_STEP in the update, OP_TCG_CHECK in the direction
// update) instead of a separate k_finalize launch; null = read the decision from the state.
hipError_t launch_tcg_dir(int r, int b, const LaunchCtx& c, const double* z, double* delta,
                          const FinalizeArgs* fin = nullptr, int* arrive = nullptr);
// Merged tCG iteration (after OP_TCG_STEP_CHECK): eta += step delta with the partial <eta_old, Hdelta>
// into c.partials slot 0; for agents that continue also r += alpha Hdelta and delta = -Prec(r) + beta delta
// (z never stored).  first: eta = 0 and r_in = grad; last: no r / delta update (tCG ends at MAXITER).
hipError_t launch_tcg_updir(int r, int b, const LaunchCtx& c, const double* X, const double* Minv, int pmode,
                            double* delta, const double* Hdelta, double* eta, const double* r_in, double* rv,
                            int first, int last);
// status_ref (optional, with g): also the partials |out - ref|^2 and |X - ref|^2 (slots 2, 3) for the status
// folded into the rho test (OptScalars::status_fold)
hipError_t launch_retract(int r, int b, const LaunchCtx& c, const double* X, const double* V, double scale,
                          double* out, const double* g, const double* HV, const double* delta_impl = nullptr,
                          const double* status_ref = nullptr);
hipError_t launch_tangent(int r, int b, const LaunchCtx& c, const double* X, const double* V, double* out);
hipError_t launch_precond(int r, int b, const LaunchCtx& c, const double* X, const double* Minv, int pmode,
                          const double* V, double* out);
// xcopy (optional): the X operand as read (PGOAgent::iterate's XPrev = X, src/PGOAgent.cpp:673)
hipError_t launch_polar_vnext(int r, int b, const LaunchCtx& c, const double* X, double* V, const double* Yv,
                              double gv, double sa, double sb, double* out, double* xcopy = nullptr);
hipError_t launch_polar_comb(int r, int b, const LaunchCtx& c, const double* A, const double* Bv,
                             const double* ca, const double* cb, double* out, const double* Cv = nullptr,
                             double sa = 1.0, double sb = 0.0, double* out2 = nullptr, double* xcopy = nullptr);
// PGOAgent::computeConvergedLoopClosureRatio (src/PGOAgent.cpp:1247-1289): per agent a, the share of
// its loop closures idx[off[a] .. off[a+1]) whose weight w[] is exactly 1 or 0 (0/0 = NaN, as there)
hipError_t launch_conv_ratio(int num_agents, const int* off, const int* idx, const double* w, double* ratio,
                             hipStream_t stream);
// partial |A - B|^2 per tile (no output vector)
hipError_t launch_sqdiff(int r, int b, const LaunchCtx& c, const double* A, const double* Bv);
hipError_t launch_select(int r, int b, const LaunchCtx& c, const double* A, const double* Bv, const int* use_a,
                         const double* ref, double* out);
hipError_t launch_accept(int r, int b, const LaunchCtx& c, const double* x2, const double* g2, const double* S2,
                         double* x1, double* g, double* S);
hipError_t launch_finalize(const FinalizeArgs& f, int num_agents, hipStream_t stream);
// exact preconditioner, one tree level of one sweep: items = (node, row block of kThreads rows) /
// (node, row tile) / (node, column tile); rhs, y, x in the engine's pose layout
hipError_t launch_sn_assemble(int r, int b, const SnView& v, const int2* items, int count, const double* rhs,
                              hipStream_t stream);
hipError_t launch_sn_fwd(int r, int b, const SnView& v, const int2* items, int count, double* y, hipStream_t stream);
// the forward sweep's items of nodes with at most kSnSmallNs S column tiles (k_sn_fwd_small)
hipError_t launch_sn_fwd_small(int r, int b, const SnView& v, const int2* items, int count, double* y,
                               hipStream_t stream);
hipError_t launch_sn_bwd(int r, int b, const SnView& v, const int2* items, int count, const double* y, double* x,
                         hipStream_t stream);
// numeric factorisation of one tree level's supernodes (count nodes, v.nodes), see SnFactorView
hipError_t launch_sn_factor(int b, const SnFactorView& v, int count, hipStream_t stream);
// the same tile-parallel over a level's nodes, one launch of the sequence (kind 0 assembly phase `param`: 0 zero,
// 1 entries, 2 + c child c; 1 diagonal tile K = param; 2 L_IK; 3 trailing F_IJ; 4 panel column J = param; 5 the
// trailing F_IJ right of the column block starting at K = param, all of the block's K at once); items:
// (node, row block / entry chunk / I / I << 16 | J)
hipError_t launch_sn_factor_tiled(int b, const SnFactorView& v, int kind, int param, const int2* items, int count,
                                  hipStream_t stream);
// z = P_X(zraw) (or z = zraw when project == 0; z = in, unprojected, for an agent with ident[agent] != 0 -- its
// factorisation failed); optional z_out / delta_out = -z; partials <z, rref>, |rref|^2 per tile
hipError_t launch_precond_finish(int r, int b, const LaunchCtx& c, const double* X, const double* zraw,
                                 const double* in, const int* ident, const double* rref, int project, double* z_out,
                                 double* delta_out);
hipError_t launch_bj_inverse(int b, int n, const QView& q, double shift, double* Minv, hipStream_t stream);
// Rebuild the edge-stream Q on device from per-edge weights w[edge] (problem edge order): records
// M = T diag(w kappa I, w tau) and packed diagonal blocks, the same arithmetic as the host build.
hipError_t launch_edge_reweight(int d, int m, int n, const double* raw, const int* slot_of_edge, const double* w,
                                const int* dinc_ptr, const int* dinc, double* wslot, double* rec, double* diag,
                                hipStream_t stream);
hipError_t launch_gnc_snapshot(int r, int b, const GncEntries& g, const double* X, const double* RX, const int* mask,
                               hipStream_t stream);
hipError_t launch_gnc_weights(int r, int b, const GncEntries& g, const double* X, const double* RX,
                              const RobustParams& rp, double* w_prob, double* w_g, hipStream_t stream);
// Lanczos helpers over flat vectors of length len: partial[g * k + j] = sum over grid block g's
// chunk of w . basis_j (fixed grid kDotBlocks, fixed order); w -= sum_j c_j basis_j (c on device)
constexpr int kDotBlocks = 512;
hipError_t launch_dot_multi(long len, const double* w, const double* basis, int k, double* partial,
                            hipStream_t stream);
hipError_t launch_axpy_multi(long len, double* w, const double* basis, int k, const double* c, hipStream_t stream);
hipError_t launch_scale(long len, const double* src, double s, double* dst, hipStream_t stream);
// dst[x * dst_stride] = src[x * src_stride], x < len (one row of the lifted layout <-> a compact vector)
hipError_t launch_strided_copy(long len, const double* src, int src_stride, double* dst, int dst_stride,
                               hipStream_t stream);
hipError_t launch_bj_inverse_diag(int b, int n, const QView& q, double shift, double* Minv, hipStream_t stream);

// ---- Jacobi-PCG on SPD block-sparse systems with several right-hand sides (GPU chordal
// initialisation, init.cpp).  Vectors are [row][bs][nr]: row p holds bs x nr doubles (column a of
// the block row is right-hand side a).  Blocks row-major bs x bs; minv: per row the inverse of the
// diagonal block.  Reductions: fixed grid kPcgBlocks, partial[block][q] then summed on the host.
constexpr int kPcgBlocks = 1024;
struct PcgCoef {
  double v[3];
};
// y = A x
hipError_t launch_pcg_spmv(int bs, int nr, int n, const int* rowptr, const int* col, const double* blk,
                           const double* x, double* y, hipStream_t stream);
// partial[block * nr + a] = sum over the block's rows of <u_a, v_a>
hipError_t launch_pcg_dot(int bs, int nr, int n, const double* u, const double* v, double* partial,
                          hipStream_t stream);
// x += alpha p, r -= alpha q, z = minv r; partial[block * 2 nr + a] = <r_a, z_a>, [.. + nr + a] = |r_a|^2
hipError_t launch_pcg_update(int bs, int nr, int n, PcgCoef alpha, const double* p, const double* q, double* x,
                             double* r, double* z, const double* minv, double* partial, hipStream_t stream);
// p = z + beta p
hipError_t launch_pcg_dir(int bs, int nr, int n, PcgCoef beta, const double* z, double* p, hipStream_t stream);

}  // namespace dpgo

/*
 * dpgo_rbcd.h -- pose-graph inputs and the multi-agent RBCD round engine (libdpgo_hip.so).
 *
 * Graph side (host C++):
 *   dpgo_graph_read_g2o      read_g2o_file            src/DPGO_utils.cpp:78-212 (+ SURVEY App. B fixes)
 *   dpgo_graph_laplacian_bsr constructConnectionLaplacianSE  src/DPGO_utils.cpp:214-286
 *   dpgo_graph_grid3d        synthetic 3D grid (replaces the missing g2o100k/1M inputs)
 *   dpgo_graph_chain_init    odometryInitialization   src/DPGO_utils.cpp:426-447, lifted by YLift
 *
 * Engine side: N PGOAgents partitioned over ranks (one process per GPU).  Per RBCD iteration
 * one colour class of the agent-adjacency graph is "selected" (doOptimization = true,
 * src/PGOAgent.cpp:642-718); all other agents run iterate(false).  Selected agents on a GPU are
 * solved as ONE batched dpgo_hip_problem (their Q blocks are independent).  Neighbour public poses
 * cross ranks either through the library's own RCCL exchange (dpgo_rbcd_comm_init / dpgo_rbcd_exchange)
 * or through caller-owned device buffers the caller moves itself (dpgo_rbcd_pack, then e.g. an RCCL
 * all_to_all, then dpgo_rbcd_update); same-rank neighbours are read directly from device memory.
 * Robust cost: L2 (default, the throughput setting) or any of the reference's RobustCostType with
 * on-device loop-closure reweighting every robust_opt_inner_iters iterations (PGOAgent::iterate +
 * updateLoopClosuresWeights, src/PGOAgent.cpp:642-718, 1174-1244; RobustCost, src/DPGO_robust.cpp).
 */
#ifndef DPGO_RBCD_H
#define DPGO_RBCD_H

#include "dpgo_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dpgo_graph_s* dpgo_graph;
typedef struct dpgo_rbcd_s* dpgo_rbcd;

/* ---- pose graphs --------------------------------------------------------------------------*/
int dpgo_graph_read_g2o(const char* path, dpgo_graph* out);
int dpgo_graph_grid3d(int k, unsigned long long seed, double rot_sigma, double trans_sigma,
                      dpgo_graph* out);
int dpgo_graph_from_arrays(int d, int n, int m, const int* p1, const int* p2, const double* R,
                           const double* t, const double* kappa, const double* tau, dpgo_graph* out);
/* d, n = max pose index + 1, m = #edges, duplicates = #repeated (p1,p2) pairs */
int dpgo_graph_info(dpgo_graph g, int* d, int* n, int* m, int* duplicates);
/* R row-major d*d per edge, t d per edge; any output may be NULL */
int dpgo_graph_copy_out(dpgo_graph g, int* p1, int* p2, double* R, double* t, double* kappa,
                        double* tau);
int dpgo_graph_destroy(dpgo_graph g);
/* Whole-graph Q as BSR (block (j, bcol) column-major).  Call with browptr == NULL to get nnzb. */
int dpgo_graph_laplacian_bsr(dpgo_graph g, long long* nnzb, int* browptr, int* bcol, double* blocks);
/* X = YLift * T_odo, T_odo composed along the p2 = p1 + 1 edges (r x (d+1) n, column-major). */
int dpgo_graph_chain_init(dpgo_graph g, int r, const double* YLift_colmajor, double* X_out);
/* chordalInitialization (src/DPGO_utils.cpp:377-424, PGOAgent::localInitialization for the L2 cost):
 * rotations by least squares with R_0 = I then projectToRotationGroup, translations by least squares
 * with t_0 = 0 (normal equations by a host block Cholesky; the reference uses SPQR, same minimiser).
 * Host-only.  T_out: d x (d+1) n column-major ([R_i | t_i] per pose); R d*d row-major per edge. */
int dpgo_chordal_initialization(int d, int n, int m, const int* p1, const int* p2, const double* R,
                                const double* t, const double* kappa, const double* tau, double* T_out);
/* X = YLift * chordal T for a graph handle (r x (d+1) n, column-major). */
int dpgo_graph_chordal_init(dpgo_graph g, int r, const double* YLift_colmajor, double* X_out);
/* chordalInitialization with both linear solves by Jacobi-preconditioned CG on the GPU (for graphs
 * whose direct factor is too large: a 10^6-pose 3D grid): each right-hand side to |r| <= rtol |b|
 * (DPGO_HIP_EDEVICE if max_iters is not enough).  iters: PCG iterations of both solves; relres: the
 * largest final relative residual.  Same system assembly and projections as the host version. */
int dpgo_chordal_initialization_gpu(int d, int n, int m, const int* p1, const int* p2, const double* R,
                                    const double* t, const double* kappa, const double* tau, double rtol,
                                    int max_iters, double* T_out, int* iters, double* relres);
int dpgo_graph_chordal_init_gpu(dpgo_graph g, int r, const double* YLift_colmajor, double rtol, int max_iters,
                                double* X_out, int* iters, double* relres);
/* The multi-robot initialisation: PGOAgent::localInitialization on every agent (chordal on its private
 * graph, src/PGOAgent.cpp:947-962; anchored at the agent's breadth-first centre pose instead of its
 * first pose -- the unconstrained rotation relaxation shrinks with graph distance from the anchor)
 * then initializeInGlobalFrame (:369-432): agents join the frame of the agent holding pose 0 in
 * breadth-first order, each by the L2 average over its shared loop closures with agents already in
 * the frame (the reference averages with GNC-TLS; identical on outlier-free data).  use_gpu: the
 * block-diagonal chordal systems by Jacobi-PCG on the device (rtol, max_iters), else host Cholesky.
 * X_out = YLift * T (r x (d+1) n, column-major). */
int dpgo_graph_distributed_init(dpgo_graph g, int num_agents, const int* agent_of_pose, int r,
                                const double* YLift_colmajor, int use_gpu, double rtol, int max_iters, double* X_out,
                                int* iters, double* relres);
/* Grid graphs: agent = sub-cube (x/s, y/s, z/s), s = k / A; id = ax + A (ay + A az). */
/* Certified optimality gap of an iterate X (r x (d+1) n, column-major, e.g. the engine's
 * dpgo_rbcd_get_X gathered over ranks) for the whole graph's central Q (unit weights): lambda_min of
 * the certificate matrix S(X) = Q - Lambda(X) (dpgo_hip_certify), f_relax = f(X), and f_rounded =
 * f of X rounded to SE(d) as PGOAgent::getTrajectoryInLocalFrame does (src/PGOAgent.cpp:481-498;
 * T_rounded: d x (d+1) n, optional; eigvec: the Ritz vector of lambda_min, r x (d+1) n, optional).
 * lambda_min >= -eps certifies f_relax <= f* <= f_rounded.
 * Not in the reference (parity-unpinned against it; pinned against the oracle's explicit S). */
int dpgo_graph_certify(dpgo_graph g, int r, const double* X, int max_iters, double tol, double* lambda_min,
                       double* residual, int* iters, double* f_relax, double* f_rounded, double* T_rounded,
                       double* eigvec);
/* The same through dpgo_hip_certify_ex (thick restart with basis_max, DPGO_CERT_SEED_X, the bound in info). */
int dpgo_graph_certify_ex(dpgo_graph g, int r, const double* X, int max_iters, int basis_max, int flags, double tol,
                          double* lambda_min, double* f_relax, double* f_rounded, double* T_rounded, double* eigvec,
                          dpgo_cert_info* info);
int dpgo_graph_grid_partition(dpgo_graph g, int agents_per_axis, int* agent_of_pose);

/* ---- RBCD engine ----------------------------------------------------------------------------*/
typedef struct {
  int r;                  /* relaxation rank */
  int acceleration;       /* Nesterov (PGOAgentParameters::acceleration) */
  int restart_interval;   /* 30 */
  int max_inner;          /* tCG iterations per update (10, src/PGOAgent.cpp:1135) */
  double initial_radius;  /* 100 (src/PGOAgent.cpp:1136) */
  double tolerance;       /* 1e-2 (src/PGOAgent.cpp:1133) */
  int precon;             /* DPGO_PRECON_BLOCK_JACOBI */
  int algorithm;          /* DPGO_ALG_RTR / DPGO_ALG_RGD */
  int q_format;           /* DPGO_QFMT_EDGES (default: edge-stream Q) or DPGO_QFMT_BSR (explicit Q) */
  /* robust cost (RobustCostParameters, include/DPGO/DPGO_robust.h; PGOAgentParameters) */
  int robust_cost;             /* DPGO_ROBUST_* (default L2) */
  int robust_opt_inner_iters;  /* 30: reweight when (iteration + 1) % this == 0 */
  int gnc_max_iters;           /* 100 */
  double gnc_barc;             /* 10 */
  double gnc_mu_step;          /* 1.4 */
  double gnc_init_mu;          /* 1e-4 */
  double huber_threshold;      /* 3 */
  double tls_threshold;        /* 10 */
  /* PGOAgent status after every selected update (src/PGOAgent.cpp:700-716): relativeChange =
   * |X - XPrev| / sqrt(n) and readyToTerminate, on the device (dpgo_rbcd_status) */
  int status;                    /* 1 (the reference always computes it) */
  double rel_change_tol;         /* 5e-3 (PGOAgentParameters::relChangeTol) */
  double min_convergence_ratio;  /* 0.8 (robustOptMinConvergenceRatio, GNC_TLS only) */
} dpgo_rbcd_params;

/* RobustCostType (include/DPGO/DPGO_robust.h): weights need an edge-stream Q (q_format EDGES) */
#define DPGO_ROBUST_L2 0
#define DPGO_ROBUST_L1 1
#define DPGO_ROBUST_TLS 2
#define DPGO_ROBUST_HUBER 3
#define DPGO_ROBUST_GM 4
#define DPGO_ROBUST_GNC_TLS 5

void dpgo_rbcd_default_params(dpgo_rbcd_params* p);
/* Host-only (no GPU needed): the public-pose exchange plan of `rank` -- poses per peer it sends /
 * receives (counts in poses) and, if the arrays are non-NULL, the global pose ids, peer-major,
 * ascending within a peer.  dpgo_rbcd_pack / all_to_all / dpgo_rbcd_update follow this plan. */
int dpgo_rbcd_plan(dpgo_graph g, int num_agents, const int* agent_of_pose, const int* agent_rank, int rank,
                   int world, long long* send_counts, long long* recv_counts, int* send_poses, int* recv_poses);
/* agent_of_pose[n] in [0, num_agents); agent_rank[num_agents] in [0, world). */
int dpgo_rbcd_create(dpgo_graph g, int num_agents, const int* agent_of_pose, const int* agent_rank,
                     int rank, int world, const dpgo_rbcd_params* p, dpgo_rbcd* out);
int dpgo_rbcd_destroy(dpgo_rbcd e);
/* Launch every engine operation on a caller-owned hipStream_t from now on (NULL = the HIP null
 * stream); work queued on the previous stream is drained first.  The engine never destroys it. */
int dpgo_rbcd_set_stream(dpgo_rbcd e, void* stream);
/* Back to the engine's own (non-blocking) stream. */
int dpgo_rbcd_reset_stream(dpgo_rbcd e);
/* number of colour classes, agents owned by this rank, poses owned by this rank */
int dpgo_rbcd_info(dpgo_rbcd e, int* num_colors, int* owned_agents, int* owned_poses,
                   int* owned_agents_per_color /* [num_colors] or NULL */);
int dpgo_rbcd_color_of_agent(dpgo_rbcd e, int* color /* [num_agents] */);
/* doubles this rank sends to / receives from each peer per exchange (world entries each) */
int dpgo_rbcd_exchange_counts(dpgo_rbcd e, long long* send_counts, long long* recv_counts);
/* global r x (d+1) n column-major host X: copy the owned poses in; (re)initialise Nesterov state */
int dpgo_rbcd_set_X(dpgo_rbcd e, const double* X_global);
/* write the owned poses into a global host array (other poses untouched) */
int dpgo_rbcd_get_X(dpgo_rbcd e, double* X_global);
/* Phase 1 of iteration with selected colour c: every non-selected agent runs iterate(false).  Any colour order:
 * a robust cost's reweighting (src/PGOAgent.cpp:1174-1244) reads the agent's own X and, for shared loop closures,
 * its neighborPoseDict -- the neighbour poses it received when it was last selected (the engine snapshots them in
 * dpgo_rbcd_update*), so results do not depend on the rank count or on the halo kind. */
int dpgo_rbcd_pre_exchange(dpgo_rbcd e, int color);
/* Pack the public poses peers need into send_dev (their X: with Nesterov the aux pose a receiver
 * uses equals the sender's X, which ran iterate(false) this iteration). */
int dpgo_rbcd_pack(dpgo_rbcd e, double* send_dev);
/* Phase 2: selected agents of colour c update from the received neighbour poses. */
/* Restrict the next updates to a subset of the selected colour's agents (agent_mask [num_agents], 1 =
 * optimise; nullptr = every agent of the colour, the colour schedule).  The others of the colour run
 * PGOAgent::iterate(false) like every other colour's agents (X = Y with acceleration, X unchanged without) and
 * do not receive neighbour poses (their reweighting keeps reading their older dictionaries), so
 * selecting one agent per round (colour = its colour) is the example's greedy schedule
 * (examples/MultiRobotExample.cpp:243-256: the next robot is the argmax of the per-robot |RieGrad|, which
 * dpgo_rbcd_central_eval returns squared per agent). */
int dpgo_rbcd_set_selected(dpgo_rbcd e, const int* agent_mask);
int dpgo_rbcd_update(dpgo_rbcd e, int color, const double* recv_dev, dpgo_opt_result* results);
/* Per-colour halo (examples/MultiRobotExample.cpp:188-213: only the selected robot pulls its neighbours'
 * poses): the poses the agents of colour c read this iteration -- about half the full plan with two
 * colours.  Same call order as the full halo: dpgo_rbcd_pre_exchange(c), dpgo_rbcd_pack_color(c) into a
 * buffer laid out by dpgo_rbcd_exchange_counts_color(c) (peer-major, ascending global pose id), the
 * exchange, dpgo_rbcd_update_color(c).  Results are bitwise those of the full halo, in any colour order and with
 * any robust cost (nothing but the selected colour reads the halo).  dpgo_rbcd_central_eval always takes the full
 * plan. */
int dpgo_rbcd_plan_color(dpgo_graph g, int num_agents, const int* agent_of_pose, const int* agent_rank, int color,
                         int rank, int world, long long* send_counts, long long* recv_counts, int* send_poses,
                         int* recv_poses);
int dpgo_rbcd_exchange_counts_color(dpgo_rbcd e, int color, long long* send_counts, long long* recv_counts);
int dpgo_rbcd_pack_color(dpgo_rbcd e, int color, double* send_dev);
int dpgo_rbcd_update_color(dpgo_rbcd e, int color, const double* recv_dev, dpgo_opt_result* results);
/* Algorithmic HBM bytes of one X.Q SpMM over colour class c on this rank, and the timed average
 * of `reps` such launches (ms, HIP events on the engine stream). */
int dpgo_rbcd_bench_spmm(dpgo_rbcd e, int color, int reps, double* bytes, double* ms);
/* Bytes of one X.Q SpMM over colour class c on this rank: SURVEY 8(d)'s B_spmm for Q as explicit
 * blocks, and the bytes of the form the engine stores (edge stream by default). */
int dpgo_rbcd_spmm_bytes(dpgo_rbcd e, int color, double* bsr_bytes, double* format_bytes);
/* Average ms of one Riemannian HVP over colour class c at the current X (HIP events). */
int dpgo_rbcd_bench_hvp(dpgo_rbcd e, int color, int reps, double* ms);
/* SpMM / HVP launches issued so far (for throughput accounting) */
int dpgo_rbcd_counters(dpgo_rbcd e, long long* agent_updates, long long* iterations);

/* Central evaluation (examples/MultiRobotExample.cpp:229-235): this rank's share of the whole-graph
 * cost f(X) = 1/2 <X Q, X> (sum over ranks = the central cost; Q is the dataset's, unit weights, as the
 * example's QCentral -- with a robust cost the reweighted Q of the solve is not what is evaluated)
 * and, per owned agent, |RieGrad|^2 of its block (the greedy selection / stop test, :243-256).
 * Call between iterations; recv_dev: the public poses of a dpgo_rbcd_pack + exchange done after the
 * last update (required when world > 1).  gradnorm_sq[num_agents]: 0 for agents of other ranks.
 * Synchronises. */
int dpgo_rbcd_central_eval(dpgo_rbcd e, const double* recv_dev, double* f_out, double* gradnorm_sq);
/* PGOAgentStatus of every owned agent's last selected update (src/PGOAgent.cpp:700-716):
 * relativeChange and readyToTerminate, written at the agent's global index (others untouched).
 * PGOAgent::shouldTerminate (:1007-1031) = every agent ready, gathered over ranks by the caller. */
int dpgo_rbcd_status(dpgo_rbcd e, double* rel_change, int* ready);
/* Cumulative solver counters per owned agent (DPGO_STATS_INTS ints at the agent's global index,
 * layout of dpgo_hip_stats). */
int dpgo_rbcd_stats(dpgo_rbcd e, int* out);
/* Algorithmic HBM bytes of every kernel the engine launched so far (SURVEY 8(d) accounting over the
 * exact per-agent launch counts) and, per colour, the bytes of one tCG-start evaluation pass
 * (k_spmm MODE_EVAL_TCG) over the colour (evaltcg_bytes_per_color[num_colors], may be NULL). */
int dpgo_rbcd_bytes(dpgo_rbcd e, double* bytes, double* evaltcg_bytes_per_color);
/* ---- native halo exchange (examples/MultiRobotExample.cpp:188-213) -------------------
 * RCCL point-to-point over the ranks of the engine, without torch: dpgo_rccl_unique_id on one rank
 * (DPGO_RCCL_ID_BYTES opaque bytes, broadcast by the caller out of band), dpgo_rbcd_comm_init on every
 * rank (collective; the engine owns and destroys the communicator), or dpgo_rbcd_comm_attach of a
 * caller-owned ncclComm_t of the same RCCL instance (its size / rank must equal world / rank).  Per
 * iteration, after dpgo_rbcd_pre_exchange: dpgo_rbcd_exchange packs the public poses and posts one
 * ncclGroupStart / per-peer ncclSend + ncclRecv / ncclGroupEnd on the engine stream; *recv_dev is the
 * engine-owned receive buffer to pass to dpgo_rbcd_update.  RCCL is resolved at run time (the copy
 * already loaded in the process, else the system librccl.so.1); DPGO_HIP_EDEVICE if absent. */
#define DPGO_RCCL_ID_BYTES 128
int dpgo_rccl_unique_id(void* id_out);
int dpgo_rbcd_comm_init(dpgo_rbcd e, const void* id);
int dpgo_rbcd_comm_attach(dpgo_rbcd e, void* comm);
/* dpgo_hip_exact_factor_info of the colour's batched problem (zeros when this rank owns none of its agents) */
int dpgo_rbcd_exact_factor_info(dpgo_rbcd e, int color, long long* nodes, int* levels, int* max_s_tiles,
                                long long* panel_doubles, double* factor_ms, int* factor_count);
/* dpgo_hip_exact_factor_flops of the colour's batched problem (zeros when this rank owns none of its agents) */
int dpgo_rbcd_exact_factor_flops(dpgo_rbcd e, int color, double* cholesky_flops, double* inverse_flops);
/* dpgo_hip_exact_sweep_bytes of the colour's batched problem (zeros when this rank owns none of its agents) */
int dpgo_rbcd_exact_sweep_bytes(dpgo_rbcd e, int color, double* fwd_bytes, double* bwd_bytes);
/* dpgo_hip_bench_precond over colour class c's batched problem, right-hand side the colour's current X */
int dpgo_rbcd_bench_precond(dpgo_rbcd e, int color, int reps, double* ms_fwd, double* ms_bwd, double* panel_bytes);
/* The engine's RCCL communicator as RCCL sees it (ncclCommCount, ncclCommUserRank); -1, -1 without one. */
int dpgo_rbcd_comm_info(dpgo_rbcd e, int* count, int* rank);
int dpgo_rbcd_exchange(dpgo_rbcd e, const double** recv_dev);
/* the per-colour halo of colour c by the same RCCL group (then dpgo_rbcd_update_color) */
int dpgo_rbcd_exchange_color(dpgo_rbcd e, int color, const double** recv_dev);
/* SpMM modes of the per-mode arrays, in this order: XQ, XQ_G, EVAL, HESS, F, EVAL_TCG, CERT, QF, HESS_QF,
 * HESS_M, HESS_QF_M (the last two: the merged tCG iteration's Hessian passes) */
#define DPGO_SPMM_MODES 11
/* Algorithmic bytes of one X.Q launch over every agent of `color`, per SpMM mode (out[DPGO_SPMM_MODES], indexed as
 * dpgo_rbcd_kernel_times; 0 for modes the engine does not launch in a step).  A launch over part of the batch (the
 * merged tCG's half-batch launches on two streams, tuning key 10) moves its share of these bytes: divide by
 * dpgo_rbcd_kernel_times_ex's full-batch equivalents, not by the launch count. */
int dpgo_rbcd_mode_bytes(dpgo_rbcd e, int color, double* out);
/* HIP events around in-step X.Q launches (on the launch stream): `period` 0 = off, 1 = every launch, k = every
 * k-th launch of each mode (a sample: an event pair adds a dispatch gap of a few microseconds around its launch);
 * dpgo_rbcd_kernel_times synchronises and returns, per SpMM mode (DPGO_SPMM_MODES entries, order above), the
 * summed milliseconds and launch counts of the timed launches since the last call. */
int dpgo_rbcd_set_kernel_timing(dpgo_rbcd e, int period);
/* dpgo_hip_problem_set_tuning on every colour problem of the engine (A/B timing on one engine). */
int dpgo_rbcd_set_tuning(dpgo_rbcd e, int key, int value);
/* Per-iteration RTR / tCG trace of every owned agent's updates (dpgo_hip_set_trace / _get_trace
 * records, per agent at its global index). */
int dpgo_rbcd_set_trace(dpgo_rbcd e, int capacity);
int dpgo_rbcd_get_trace(dpgo_rbcd e, int agent, double* out, int max_records, int* count);
int dpgo_rbcd_kernel_times(dpgo_rbcd e, double* ms_per_mode, long long* launches_per_mode);
/* dpgo_rbcd_kernel_times plus, per mode, the timed launches' summed share of their batch's tiles (full-batch launch
 * equivalents: a launch over every agent counts 1, a half-batch launch about 0.5); any pointer may be null. */
int dpgo_rbcd_kernel_times_ex(dpgo_rbcd e, double* ms_per_mode, long long* launches_per_mode, double* batch_equiv);

#ifdef __cplusplus
}
#endif
#endif /* DPGO_RBCD_H */

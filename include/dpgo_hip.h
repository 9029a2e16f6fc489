/*
 * dpgo_hip.h -- C ABI of the MI355X-native DPGO RBCD hot path (libdpgo_hip.so).
 *
 * This is the drop-in boundary that sits under the reference's C++ API
 * (QuadraticProblem / QuadraticOptimizer / LiftedSEManifold / PGOAgent::updateX).
 * Every entry point cites the reference interface it replaces (paths relative to the
 * lajoiepy/dpgo source root).  The C++ shim classes in dpgo_amd/cpp keep the reference
 * signatures and forward here; INTEGRATION.md shows the binding a maintainer would add.
 *
 * Conventions
 *  - All arithmetic is fp64.  d in {2,3}, b = d+1, r = relaxation rank, 2 <= r <= 8, r >= d.
 *  - Pose matrices use the reference layout: X is r x (b n), column-major, so pose j is the
 *    contiguous r*b doubles [Y_j (r x d, col-major) | p_j (r)]   (tests/testEigenMap.cpp:19-35).
 *  - A problem handle holds one or more *agents* (independent RBCD blocks) whose poses are
 *    concatenated in agent order; single-agent handles reproduce QuadraticProblem exactly.
 *    Per-agent outputs (f, norms, results) are arrays of length num_agents.
 *  - Host-pointer entry points copy in/out and synchronise; *_dev entry points take device
 *    pointers, run asynchronously on the handle's stream and never synchronise unless stated.
 *  - Return value: 0 (DPGO_HIP_OK) or a negative error code; dpgo_hip_last_error() returns a
 *    thread-local message.  No C++ exception crosses this boundary.  There is no CPU fallback:
 *    without a usable gfx950 device every compute call returns DPGO_HIP_ENODEV.
 */
#ifndef DPGO_HIP_H
#define DPGO_HIP_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DPGO_HIP_OK 0
#define DPGO_HIP_EINVAL (-1)
#define DPGO_HIP_ENODEV (-2)
#define DPGO_HIP_EDEVICE (-3)
#define DPGO_HIP_ENOMEM (-4)
#define DPGO_HIP_ESTATE (-5)

/* Preconditioner modes (QuadraticProblem::PreConditioner, src/QuadraticProblem.cpp:75-87).
 * EXACT: the reference's own -- P_X(V (Q + 0.1 I)^-1) with a supernodal multifrontal Cholesky factor of
 * Q + 0.1 I: nested-dissection tree built on the host once per Q pattern, numeric factorisation on the GPU for an
 * edge-stream Q (per tree level, dense frontal tiles on the fp64 matrix cores; again after every on-device
 * reweighting) or on the host for a BSR Q; each application is two sweeps of dense panel products
 * [L_SS^-1 ; L_RS L_SS^-1] per supernode, one launch per tree level and sweep.  If Q + 0.1 I is not positive
 * definite it falls back to the identity, as the reference does (:81-86).
 * BLOCK_JACOBI: per-pose (Q_jj + 0.1 I)^-1 (the north_star's throughput choice). NONE: identity. */
#define DPGO_PRECON_EXACT 0
#define DPGO_PRECON_BLOCK_JACOBI 1
#define DPGO_PRECON_NONE 2

/* Device form of Q: explicit block-sparse rows, or the measurement (edge) stream it is built from */
#define DPGO_QFMT_BSR 0
#define DPGO_QFMT_EDGES 1

/* ROPTALG (include/DPGO/DPGO_types.h:29-35) */
#define DPGO_ALG_RTR 0
#define DPGO_ALG_RGD 1

/* ROPTLIB tCGstatusSet */
#define DPGO_TCG_NEGCURVTURE 0
#define DPGO_TCG_EXCREGION 1
#define DPGO_TCG_LCON 2
#define DPGO_TCG_SCON 3
#define DPGO_TCG_MAXITER 4

typedef struct dpgo_hip_problem_s* dpgo_hip_problem;

/* QuadraticOptimizer setters (include/DPGO/QuadraticOptimizer.h:34-71, defaults
 * src/QuadraticOptimizer.cpp:20-30) plus the preconditioner mode. */
typedef struct {
  int algorithm;             /* DPGO_ALG_RTR / DPGO_ALG_RGD */
  double rgd_stepsize;       /* setGradientDescentStepsize (1e-3) */
  int tr_iterations;         /* setTrustRegionIterations (1) */
  double tr_tolerance;       /* setTrustRegionTolerance (1e-2) */
  double tr_initial_radius;  /* setTrustRegionInitialRadius (10) */
  int tr_max_inner;          /* setTrustRegionMaxInnerIterations (50) */
  int verbose;               /* setVerbose */
  int precon;                /* DPGO_PRECON_* (BLOCK_JACOBI) */
} dpgo_opt_params;

/* ROPTResult (include/DPGO/DPGO_types.h:40-59) + solver counters */
typedef struct {
  int success;
  double fInit, gradNormInit, fOpt, gradNormOpt, relativeChange, elapsedMs;
  int tCGStatus;      /* DPGO_TCG_* of the last tCG, -1 if no tCG ran */
  int runs;           /* RTR Run() calls (radius-shrink retries) */
  int outer_iters;    /* RTR outer iterations */
  int inner_iters;    /* tCG iterations of the last tCG */
  int gave_up;        /* "Too many RTR rejections" (returned the input) */
} dpgo_opt_result;

/* ---- library ---------------------------------------------------------------------------*/
const char* dpgo_hip_version(void);
const char* dpgo_hip_last_error(void);
/* Number of usable gfx950 devices (0 if none). */
int dpgo_hip_device_count(void);
void dpgo_hip_default_params(dpgo_opt_params* p);

/* ---- problem lifecycle (QuadraticProblem ctor/dtor, src/QuadraticProblem.cpp:16-29) ----*/
int dpgo_hip_problem_create(int n, int d, int r, dpgo_hip_problem* out);
/* num_agents independent blocks with poses_per_agent[a] poses each (batched RBCD). */
int dpgo_hip_problem_create_batch(int num_agents, const int* poses_per_agent, int d, int r,
                                  dpgo_hip_problem* out);
int dpgo_hip_problem_destroy(dpgo_hip_problem h);
/* Launch on a caller-owned hipStream_t (NULL = the handle's own stream). */
int dpgo_hip_problem_set_stream(dpgo_hip_problem h, void* stream);
int dpgo_hip_problem_info(dpgo_hip_problem h, int* num_agents, int* total_poses, int* d, int* r);
int dpgo_hip_set_precon(dpgo_hip_problem h, int mode);

/* ---- problem data ------------------------------------------------------------------------*/
/* QuadraticProblem::setQ (src/QuadraticProblem.cpp:31-42): Q of one agent in the reference's
 * Eigen RowMajor CSR (include/DPGO/DPGO_types.h:23), (b n_a) x (b n_a), int32 indices. */
int dpgo_hip_set_Q_csr(dpgo_hip_problem h, int agent, int nrows, const int* rowptr,
                       const int* colidx, const double* vals);
/* Same data as block-sparse rows: block (j, colidx[k]) stored column-major (b*b doubles).
 * nbrows == n_a; column indices are agent-local pose indices. */
int dpgo_hip_set_Q_bsr(dpgo_hip_problem h, int agent, int nbrows, const int* browptr,
                       const int* bcolidx, const double* blocks);
/* Q of one agent given by the measurements it is built from, never materialised:
 * Q = A Omega A^T (constructConnectionLaplacianSE, src/DPGO_utils.cpp:214-286) for private edges,
 * plus the diagonal terms of shared edges (PGOAgent::constructQMatrix, src/PGOAgent.cpp:720-781).
 * m edges with agent-local endpoints p1 -> p2; an endpoint of -1 marks a shared edge whose other
 * end lives in another agent (it then adds T Omega T^T to Q_p1p1, or Omega to Q_p2p2, only).
 * R: d*d row-major per edge, t: d per edge, kappa/tau: precisions, weight: NULL = 1 (GNC weight w
 * multiplies both precisions).  The X.Q kernels then stream one 14-double record per edge
 * (8 for d = 2) instead of two b x b off-diagonal blocks plus diagonal blocks.  Every agent of a
 * handle must use the same form (BSR via set_Q_csr/_bsr, or edges). */
int dpgo_hip_set_Q_edges(dpgo_hip_problem h, int agent, int m, const int* p1, const int* p2,
                         const double* R, const double* t, const double* kappa, const double* tau,
                         const double* weight);
/* Reweight an edge-stream Q on the device (PGOAgent::constructQMatrix after a GNC weight update,
 * src/PGOAgent.cpp:720-781, 1181-1244): w_dev[e] (device, one weight per edge, agents' set_Q_edges
 * lists concatenated in agent order) replaces each edge's weight; records, diagonal blocks and the
 * block-Jacobi inverses are rebuilt by kernels (bitwise the host build with those weights), the
 * exact factor is refreshed on its next use.  Asynchronous on the handle's stream; w_dev must stay
 * valid until the next EXACT-preconditioned call. */
int dpgo_hip_set_edge_weights_dev(dpgo_hip_problem h, const double* w_dev);
/* QuadraticProblem::setG (src/QuadraticProblem.cpp:44-48) in sparse form: count pose blocks
 * (r x b column-major) at agent-local poses pose_idx[]; all other columns of G are zero. */
int dpgo_hip_set_G(dpgo_hip_problem h, int agent, int count, const int* pose_idx,
                   const double* blocks);
/* Dense r x (b n_a) G for one agent (column-major). */
int dpgo_hip_set_G_dense(dpgo_hip_problem h, int agent, const double* G);

/* ---- evaluations (QuadraticProblem, src/QuadraticProblem.cpp:50-101) ---------------------*/
/* f(X) = 0.5 <XQ, X> + <X, G> per agent (:50-60) */
int dpgo_hip_f(dpgo_hip_problem h, const double* X, double* f_out);
/* EucGrad: X Q + G (:62-66) */
int dpgo_hip_egrad(dpgo_hip_problem h, const double* X, double* EG);
/* EucHessianEta: V Q (:68-73) */
int dpgo_hip_ehvp(dpgo_hip_problem h, const double* V, double* HV);
/* RieGrad / RieGradNorm (:89-101): P_X(XQ + G), per-agent Frobenius norms; f_out optional */
int dpgo_hip_riegrad(dpgo_hip_problem h, const double* X, double* RG, double* norms,
                     double* f_out);
/* Riemannian Hessian at X applied to tangent V (ROPTLIB HessianEta = EucHessianEta + EucHvToHv) */
int dpgo_hip_rhvp(dpgo_hip_problem h, const double* X, const double* V, double* HV);
/* PreConditioner (:75-87) with the handle's mode */
int dpgo_hip_precondition(dpgo_hip_problem h, const double* X, const double* V, double* out);

/* ---- manifold (LiftedSEManifold / ROPTLIB Stiefel Set3), stateless ----------------------*/
/* ProductManifold::Projection: V_Y - Y sym(Y^T V_Y), V_p */
int dpgo_hip_tangent_project(int r, int d, int n, const double* X, const double* V, double* out);
/* QF retraction of scale*V at X: [qf(Y + s V_Y) | p + s V_p] */
int dpgo_hip_retract_qf(int r, int d, int n, const double* X, const double* V, double scale,
                        double* out);
/* LiftedSEManifold::project (src/manifold/LiftedSEManifold.cpp:34-45) */
int dpgo_hip_project_polar(int r, int d, int n, const double* in, double* out);

/* ---- optimisation (QuadraticOptimizer::optimize, src/QuadraticOptimizer.cpp:34-149) -----*/
/* Runs every agent of the handle; results[num_agents].  agent_enabled (optional, device or
 * host per variant) skips agents (their X_out = X_in, result.success = 0). */
int dpgo_hip_optimize(dpgo_hip_problem h, const dpgo_opt_params* params, const double* X_in,
                      double* X_out, dpgo_opt_result* results);

/* ---- device-pointer variants (asynchronous on the handle's stream) -----------------------*/
int dpgo_hip_f_dev(dpgo_hip_problem h, const double* X, double* f_out_host);
int dpgo_hip_egrad_dev(dpgo_hip_problem h, const double* X, double* EG);
int dpgo_hip_ehvp_dev(dpgo_hip_problem h, const double* V, double* HV);
int dpgo_hip_riegrad_dev(dpgo_hip_problem h, const double* X, double* RG);
int dpgo_hip_rhvp_dev(dpgo_hip_problem h, const double* X, const double* V, double* HV);
int dpgo_hip_project_polar_dev(dpgo_hip_problem h, const double* in, double* out);
/* out = project(ca[a] * A + cb[a] * B) per agent a (Nesterov updateY / updateV,
 * src/PGOAgent.cpp:1075-1091); ca/cb host arrays[num_agents]. */
int dpgo_hip_polar_combine_dev(dpgo_hip_problem h, const double* A, const double* B,
                               const double* ca, const double* cb, double* out);
/* Synchronises once per RTR Run (radius-shrink bookkeeping); results host array (may be NULL). */
int dpgo_hip_optimize_dev(dpgo_hip_problem h, const dpgo_opt_params* params, const double* X_in,
                          double* X_out, const int* agent_enabled_host, dpgo_opt_result* results);
/* Device buffer of the last tCG / RTR scalar state (for profiling / tests) */
int dpgo_hip_synchronize(dpgo_hip_problem h);

/* ---- solver statistics and per-iteration trace --------------------------------------------
 * Cumulative per-agent counters since the handle was created, DPGO_STATS_INTS ints per agent:
 * [optimize calls, calls that returned at once (|grad| < tol), RTR Runs, tCG inner iterations,
 *  tCG exits NEGCURVTURE, EXCREGION, LCON, SCON, MAXITER, updates that gave up, tCG CG steps,
 *  Runs whose tCG ended at its first step on the trust-region boundary, Runs whose first step test
 *  was the full pass that also stores Hess[delta] (chosen when the previous call took CG steps)]. */
#define DPGO_STATS_INTS 13
int dpgo_hip_stats(dpgo_hip_problem h, int* out /* [num_agents * DPGO_STATS_INTS] */);
/* Per-iteration RTR / tCG trace (the reference prints it with ROPTLIB Debug = ITERRESULT when
 * verbose, src/QuadraticOptimizer.cpp:82-86): after this call every tCG step test, tCG stopping
 * test and rho test appends one record of DPGO_TRACE_WIDTH doubles per agent, up to `capacity`
 * records per agent (0 turns tracing off).  Record fields (kernels.h TraceField): op (3 step test,
 * 4 stopping test, 5 rho test), j, f1, f2, rho, Delta, alpha, beta, tau, <delta, H delta>, |r|,
 * <z, r>, tCG status (-1 if none), accepted, |grad(x1)|, Run index. */
#define DPGO_TRACE_WIDTH 16
int dpgo_hip_set_trace(dpgo_hip_problem h, int capacity);
/* Copies agent's records (at most max_records) into out; *count = records written since
 * set_trace (may exceed capacity: the later ones were dropped). */
int dpgo_hip_get_trace(dpgo_hip_problem h, int agent, double* out, int max_records, int* count);

/* Source hash the library was compiled from (sha256 of the sources, hex; "unknown" if built
 * without it): lets a caller check that a shipped binary matches the tree it runs with. */
const char* dpgo_hip_build_id(void);

/* ---- certification (not in the reference: parity is pinned against a sparse
 * eigensolver on the explicitly formed matrix) --------------------------------------------------
 * Smallest eigenvalue of the certificate matrix S(X) = Q - Lambda(X), Lambda = blockdiag of
 * [sym(Y_j^T (XQ + G)_Y) 0; 0 0]: X is a global minimiser of the rank-r relaxation iff S(X) >= 0.
 * Lanczos with full re-orthogonalisation on the device (the operator V -> V S(X) on r x (d+1) n
 * matrices has S's spectrum), stopping when the Ritz residual <= tol * |lambda|_max-estimate or
 * after max_iters steps.  Single-agent handles.  eigvec (host, r x (d+1) n, optional): the Ritz
 * vector of lambda_min. */
int dpgo_hip_certify(dpgo_hip_problem h, const double* X, int max_iters, double tol, double* lambda_min,
                     double* residual, int* iters, double* eigvec);
/* The same with a thick restart and a seed block.  basis_max > 0: at most basis_max Krylov vectors; a full
 * basis restarts from its lowest max(basis_max / 4, 8) Ritz vectors and the newest Krylov direction
 * (Rayleigh-Ritz on the dense projected matrix); max_iters counts operator applications over all
 * restarts.  flags DPGO_CERT_SEED_X: the principal directions of X's rows (S(X) X^T ~ 0 at a critical
 * point: the near-null space; singular values >= 1e-3 of the largest) and the translation gauge (every
 * translation column = 1, an exact null vector), orthonormalised, form a locked block U; the chain runs on its complement and U's block is
 * resolved exactly, S = [A_s B^T; B C] in (U, U_perp).  Everything lives on row 0 of the lifted layout
 * (the operator acts row by row).  lambda_min = the lowest Ritz value found (an upper bound of
 * lambda_min(S)); info (optional) carries the true residual of the returned pair and the bound
 * lower_bound = (a + c) / 2 - sqrt(((c - a) / 2)^2 + |B|_F^2), a = lambda_min(A_s), c = theta_C -
 * residual_C (the smallest eigenvalue of [a -|B|; -|B| c], which bounds x^T S x from below), rigorous when
 * theta_C is C's lowest eigenvalue to within its residual (Lanczos from a random start: with
 * probability ~1). */
#define DPGO_CERT_SEED_X 1
typedef struct {
  int iters;                  /* operator applications (all restarts) */
  int restarts;
  int seeds;                  /* independent rows of X in the locked block */
  double residual;            /* |S y - lambda_min y| of the returned Ritz pair */
  double lambda_seed;         /* lambda_min(U^T S U) (NaN without seeds) */
  double lambda_complement;   /* the chain's lowest Ritz value theta_C */
  double residual_complement; /* |P S y - theta_C y|, P = I - U U^T: its residual on C */
  double coupling;            /* |(I - U U^T) S U|_F (0 without seeds) */
  double lower_bound;         /* see above (theta_C - residual_C without seeds) */
  double ritz[8];             /* the chain's lowest Ritz values (NaN-padded) */
} dpgo_cert_info;
int dpgo_hip_certify_ex(dpgo_hip_problem h, const double* X, int max_iters, int basis_max, int flags, double tol,
                        double* lambda_min, double* eigvec, dpgo_cert_info* info);

/* ---- measurement helpers ----------------------------------------------------------------*/
/* Select a compiled kernel variant / host sequence for A/B timing (process-wide; every setting gives
 * results within the documented bars, most bitwise the default's).  key 0: BSR X.Q SpMM
 * neighbour-loop variant 0 = 1 neighbour/step (default), 1 = same with non-temporal block loads,
 * 2 = 2 neighbours/step, 3 = 4 neighbours/step, 4 = 4 + XCD-aware tile remap, 5 = 2 + XCD remap,
 * 6 = 1 + XCD remap.  key 1: edge-stream variant for every SpMM mode (same numbering over
 * incidences; -1 = the compiled default).  key 2: epilogue operands ahead of the edge loop (1, default).
 * key 3: consumer-side tCG finalize (classic sequence).  key 4: first tCG step kind (0 predicted,
 * 1 each-edge-once pass, 2 full pass).  key 5: 1 = the classic five-launch tCG iteration instead of the
 * merged one.  key 6: 1 = HESS_M operands prefetched.  key 7: tCG queueing (0 adaptive, 1 one iteration
 * ahead, 2 all at once; the classic sequence of the exact preconditioner queues all at once only with 2).  key 8: 1 = second-visit record staging (set before Q).  key 9: 1 = the agent
 * status by its own pass instead of folded into the rho test.  key 10: merged tCG iterations of a small
 * batch (<= 4,096 tiles) in two agent halves on two streams (1, default; 0 off; 2 the halves out of phase).
 * DESIGN.md records each key's measurement.  These are the process DEFAULTS: a handle copies them when it is
 * created, so handles created afterwards follow; dpgo_hip_problem_set_tuning changes one existing handle. */
int dpgo_hip_set_tuning(int key, int value);
/* The exact preconditioner's factor of the handle (after a solve that used it): supernodes, tree levels, the
 * widest separator in 64-row tiles, panel doubles, and the last device factorisation's time (ms, 0 when it ran on
 * the host) with the number of device factorisations so far. */
int dpgo_hip_exact_factor_info(dpgo_hip_problem h, long long* nodes, int* levels, int* max_s_tiles,
                               long long* panel_doubles, double* factor_ms, int* factor_count);
/* Flop counts of one numeric factorisation of that factor (the roofline of dpgo_hip_exact_factor_info's factor_ms):
 * the classic supernodal Cholesky count sum_nodes s^3/3 + s^2 t + s t^2 (s, t = the node's S and R scalars; the
 * work CHOLMOD does for src/QuadraticProblem.cpp:37-41), and the extra flops of the panels' inverse blocks
 * [L_SS^-1; L_RS L_SS^-1] (s^3/3 + s^2 t per node) that make the solves dense products.  Zeros before a factor. */
int dpgo_hip_exact_factor_flops(dpgo_hip_problem h, double* cholesky_flops, double* inverse_flops);
/* The agents of the handle whose last exact factorisation met a non-positive pivot: QuadraticProblem::PreConditioner's
 * "Preconditioner failed" branch (src/QuadraticProblem.cpp:81-86) applies to them alone -- their output is their input,
 * unprojected -- while the batch's other agents keep their factors.  flags (K ints, may be null) receives 1 per such
 * agent, *count their number (0 before any factor).  Waits for the handle's stream. */
int dpgo_hip_exact_fallback_agents(dpgo_hip_problem h, int* flags, int* count);
/* The exact preconditioner's two sweeps over every agent of the handle (right-hand side V_dev, the handle's layout),
 * `reps` applications after 3 untimed ones, each timed with HIP events on the handle's stream: the forward sweep
 * (every level's k_sn_assemble + k_sn_fwd) and the backward sweep (every level's k_sn_bwd), ms per application, and
 * the bytes of the stored panel tiles (64 x 64, padding included). */
int dpgo_hip_bench_precond(dpgo_hip_problem h, const double* V_dev, int reps, double* ms_fwd, double* ms_bwd,
                           double* panel_bytes);
/* The panel bytes one application's sweeps read: every wide supernode's 64 x 64 tiles (padding included) and the
 * compact copy of every narrow one (at most 2 S column tiles: the backward sweep always, the forward sweep on levels
 * of narrow nodes only).  Zeros before a factor. */
int dpgo_hip_exact_sweep_bytes(dpgo_hip_problem h, double* fwd_bytes, double* bwd_bytes);
/* The process default of a tuning key. */
int dpgo_hip_get_tuning(int key, int* value);
/* The same keys on one existing handle (A/B timing of variants on one problem without rebuilding it). */
int dpgo_hip_problem_set_tuning(dpgo_hip_problem h, int key, int value);
/* Algorithmic HBM bytes of one X.Q SpMM over this handle: BSR blocks + indices + X + Y, or, for
 * an edge-stream Q, every edge record once + 8 B per incidence + pointers + X + Y. */
double dpgo_hip_spmm_bytes(dpgo_hip_problem h);
/* SURVEY 8(d)'s algorithmic bytes of one X.Q SpMM over this handle's Q as explicit b x b blocks
 * (B_spmm = nnzb (b^2 8 + 4) + (n + 1) 4 + 2 r b n 8), whatever form the handle stores it in. */
double dpgo_hip_spmm_bytes_bsr(dpgo_hip_problem h);
/* Riemannian HVP timing: one EVAL at X_dev (S and the Riemannian gradient into V_dev), then `reps`
 * back-to-back Hessian-vector products HV_dev = Hess f(X)[V]; average ms per product in *ms. */
int dpgo_hip_bench_hvp(dpgo_hip_problem h, const double* X_dev, double* V_dev, double* HV_dev, int reps, double* ms);
/* Time `reps` back-to-back X.Q SpMM launches with HIP events on the handle's stream; returns the
 * average milliseconds per launch in *ms. */
int dpgo_hip_bench_spmm(dpgo_hip_problem h, const double* X_dev, double* Y_dev, int reps, double* ms);

#ifdef __cplusplus
}
#endif
#endif /* DPGO_HIP_H */

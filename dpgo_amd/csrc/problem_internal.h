// Internal (non-ABI) view of a dpgo_hip_problem, shared by capi.cpp and rbcd.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <string>
#include <vector>

#include "../../include/dpgo_hip.h"
#include "kernels.h"

namespace dpgo {

int fail(int code, const std::string& msg);
int usable_devices();

// Debug runs (DPGO_POISON=1): every fresh device allocation, and the exact preconditioner's frontal / panel /
// sweep buffers before each factorisation and application, are filled with 0xFF bytes -- a NaN in every double --
// so a kernel that reads an entry nothing wrote yields NaN instead of a plausible stale value.
bool poison_enabled();
hipError_t poison_fill(void* p, size_t bytes, hipStream_t stream);

#define HIP_TRY(expr)                                                                        \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess)                                                                    \
      return ::dpgo::fail(DPGO_HIP_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

#define DPGO_TRY(expr)                  \
  do {                                  \
    int _rc = (expr);                   \
    if (_rc != DPGO_HIP_OK) return _rc; \
  } while (0)

struct HostBSR {
  std::vector<int> rowptr, col;
  std::vector<double> blocks;
};

// One agent's Q as its measurement stream (QFMT_EDGES): agent-local endpoints (-1 = the endpoint
// lives in another agent), R (d*d row-major), t (d), and the weighted precisions w kappa, w tau.
struct HostEdges {
  std::vector<int> p1, p2;
  std::vector<double> R, t, kw, tw, kappa0, tau0;  // kw = w kappa0, tw = w tau0
};

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  unsigned alloc_flags = 0;  // hipExtMallocWithFlags flags (e.g. hipDeviceMallocContiguous); hipMalloc if it fails
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  hipError_t ensure(size_t count) {
    if (count <= n && p) return hipSuccess;
    release();
    n = std::max<size_t>(count, 1);
    hipError_t e = hipErrorMemoryAllocation;
    if (alloc_flags != 0) {
      e = hipExtMallocWithFlags(reinterpret_cast<void**>(&p), n * sizeof(T), alloc_flags);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        p = nullptr;
      }
    }
    if (e != hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&p), n * sizeof(T));
    if (e != hipSuccess || !poison_enabled()) return e;
    const hipError_t f = poison_fill(p, n * sizeof(T), nullptr);
    return f != hipSuccess ? f : hipDeviceSynchronize();
  }
};

}  // namespace dpgo

struct dpgo_hip_problem_s {
  int K = 0, d = 0, r = 0, b = 0;
  int tuning[dpgo::TUNE_COUNT] = {};  // this handle's tuning keys (the process defaults at creation)
  long N = 0;  // total poses
  std::vector<int> n_agent;
  std::vector<long> pose_off;
  hipStream_t stream = nullptr;
  hipStream_t own_stream = nullptr;

  // tiles
  std::vector<int> h_tile_agent, h_tile_start, h_tile_count, h_agent_tile_off;
  int num_tiles = 0;
  dpgo::DevBuf<int> tile_agent, tile_start, tile_count, agent_tile_off, agent_np, enabled, use_a;

  // Q (per-agent host copies, concatenated on upload)
  std::vector<dpgo::HostBSR> q_agent;
  std::vector<dpgo::HostEdges> e_agent;
  std::vector<int> q_fmt;  // per agent: QFMT_BSR / QFMT_EDGES
  int fmt = 0;             // format of the uploaded Q (all agents agree)
  bool q_dirty = true;
  dpgo::DevBuf<int> rowptr, col;
  dpgo::DevBuf<double> blocks, minv;
  long nnzb = 0;
  dpgo::DevBuf<int> inc_ptr, rec_first;
  dpgo::DevBuf<int2> inc;
  // second-visit staging: per tile the sorted ids of its second-visit edges (sv_ptr / sv_ids) and the
  // incidences with tile-local record slots (inc_sv: second visits 0.., first visits after them)
  dpgo::DevBuf<int> sv_ptr, sv_ids;
  dpgo::DevBuf<int2> inc_sv;
  dpgo::DevBuf<double> rec, diag;
  long nnz_inc = 0, num_edges = 0;
  // on-device reweighting (dpgo_hip_set_edge_weights_dev): unweighted measurement per record slot
  // [R | t | kappa | tau], problem edge -> slot, and per pose every incident edge incl. shared ones
  // (slot * 2 + (pose == p1)) in edge order, for the diagonal blocks
  dpgo::DevBuf<double> raw, wslot;
  dpgo::DevBuf<int> slot_of_edge, dinc_ptr, dinc;
  bool host_weights_stale = false;
  const double* w_dev_last = nullptr;  // caller's weight array of the last device reweighting

  // G (sparse pose blocks per agent)
  std::vector<std::map<int, std::vector<double>>> g_agent;
  bool g_dirty = true;
  dpgo::DevBuf<int> gidx;
  dpgo::DevBuf<double> gblk;
  int num_gslots = 0;

  int precon = DPGO_PRECON_BLOCK_JACOBI;

  // exact preconditioner: supernodal Cholesky of Q + 0.1 I (chol.cpp), one launch per tree level and sweep
  int chol_state = 0;  // 0 stale, 1 ready, 2 Q + 0.1 I not positive definite (identity, as the reference)
  dpgo::DevBuf<double> sn_panel, sn_F, sn_U;
  dpgo::DevBuf<long> sn_panel_off, sn_f_off, sn_u_off;
  dpgo::DevBuf<int> sn_s, sn_t, sn_poses_off, sn_poses, sn_cpos_off, sn_cpos;
  dpgo::DevBuf<int2> sn_contrib, sn_items;
  dpgo::DevBuf<int> sn_node_agent;  // [nodes] batch agent of each supernode (per-agent skip in the sweeps)
  struct SnLevel {  // item ranges into sn_items of one tree depth
    int asm0 = 0, asm_n = 0, fws0 = 0, fws_n = 0, fwd0 = 0, fwd_n = 0, bwd0 = 0, bwd_n = 0;  // fws: k_sn_fwd_small's
  };
  std::vector<SnLevel> sn_levels;  // index = depth (0 = the roots)
  // narrow supernodes' compact panels (SnView::cpanel): per node its offset (-1: tiles only), the copy's items
  // (node, 64-row block) for launch_sn_compact after every factorisation, and the bytes a sweep then reads
  dpgo::DevBuf<double> sn_cpanel;
  dpgo::DevBuf<long> sn_cpanel_off;
  dpgo::DevBuf<int2> sn_citems;
  dpgo::DevBuf<dpgo::SnItem> sn_desc;  // [items] per sweep item its node's record (SnView::desc)
  int sn_citems_n = 0;
  bool sn_compact = false;
  double sn_sweep_bytes_fwd = 0.0, sn_sweep_bytes_bwd = 0.0;
  long chol_doubles = 0;
  dpgo::DevBuf<int4> tile_meta;
  // edge-stream records and diagonal blocks at unit weights (kept by the engine under a robust cost): the central
  // evaluation of examples/MultiRobotExample.cpp:229-235 reads the dataset's Q, not the reweighted one
  dpgo::DevBuf<double> rec_unit, diag_unit;
  bool central_unit = false;  // qview() serves rec_unit / diag_unit  // edge-stream Q: per tile stage ranges (LaunchCtx::tile_meta); empty otherwise
  long sn_nodes = 0;             // supernodes of the current symbolic structure (sn_s may be larger: capacity)
  // DPGO_PANEL_GUARD (debug runs): (offset, doubles) of the NaN gap after every supernode's panel and after the last
  std::vector<std::pair<long, long>> sn_guards;
  double chol_flops = 0.0;       // the factorisation's classic flop count: sum over supernodes s^3/3 + s^2 t + s t^2
  double chol_inv_flops = 0.0;   // the panels' extra: L_SS^-1 (s^3/3) and L_RS L_SS^-1 (s^2 t) per supernode
  // device numeric factorisation (TUNE_DEVICE_CHOL, edge-stream Q): the symbolic structure is built once per Q
  // pattern (sn_sym_ready); every refresh after a reweighting re-runs only k_sn_factor, level by level
  bool sn_sym_ready = false;
  std::vector<int> fac_level_off;  // [depth + 1] into fac_nodes
  dpgo::DevBuf<int> fac_nodes, fac_ch_off, fac_ch, fac_tp_off, fac_tp, fac_ent_off, fac_src;
  // [K] per agent: 1 = its factorisation met a non-positive pivot (identity preconditioner for that agent only,
  // src/QuadraticProblem.cpp:81-86); written by the device factor, or uploaded by the host factorisation
  dpgo::DevBuf<int> fac_not_pd;
  dpgo::DevBuf<long> fac_off;
  dpgo::DevBuf<dpgo::SnEntry> fac_ent;
  dpgo::DevBuf<double> fac_F[2];  // frontal matrices of the even / odd tree depths
  // tree levels factorised tile-parallel (few, large supernodes): per depth the launch sequence of
  // launch_sn_factor_tiled over fac_titems (empty: one workgroup per node, k_sn_factor)
  struct FacLaunch {
    int kind, param, off, count;
  };
  std::vector<std::vector<FacLaunch>> fac_seq;
  dpgo::DevBuf<int2> fac_titems;
  double chol_factor_ms = 0.0;    // the last device factorisation (hipEvent), for the benches
  bool chol_factor_pending = false;  // fac_ev holds a factorisation whose time is not yet in chol_factor_ms
  int chol_factor_count = 0;
  // host copy of the edge-stream incidences (sync_q_edges), for the factor's assembly tables
  std::vector<int> h_inc_ptr;
  std::vector<int2> h_inc;

  // work
  dpgo::DevBuf<double> x1, x2, g, g2, S, S2, eta, rv, z, delta, Hdelta, tA, tB;
  dpgo::DevBuf<double> pa, pb, sums, coef_a, coef_b;
  // |X_out - X_in|^2 partials of the single-Run output select: each tile written once, in the Run
  // its agent's outcome was decided (an in-place X_in is overwritten by then)
  dpgo::DevBuf<double> pc;
  dpgo::DevBuf<double> peh;  // merged tCG: k_tcg_updir's <eta_old, Hdelta> partials (FinalizeArgs::pc)
  // TUNE_SPLIT_STREAMS: agent groups 1.. of the merged tCG iterations run on split_stream[g - 1], forked
  // from / joined into the launch stream by events
  static constexpr int kMaxSplit = 8;
  hipStream_t split_stream[kMaxSplit - 1] = {};
  hipEvent_t split_fork = nullptr, split_join[kMaxSplit - 1] = {};
  dpgo::DevBuf<dpgo::AgentState> state;
  std::vector<dpgo::AgentState> h_state;
  // per-agent arrival counts of a k_spmm with a fused finalize (0 between launches)
  dpgo::DevBuf<int> arrive;
  // finalize after an SpMM: 0 separate k_finalize launch, 1 / 2 fused into the SpMM's last block per
  // agent (SpmmArgs::fin_mode); DPGO_FUSE_FINALIZE overrides
  int fuse_finalize = 0;
  // host-mapped status words written by k_finalize (zero-copy polling, no stream sync)
  int* pub_host = nullptr;
  int* pub_dev = nullptr;
  int pub_tag = 0;
  // the first tCG step of the previous optimize call stopped every agent on the trust-region
  // boundary (or negative curvature): the next call's first step evaluates only <delta, Hess delta>
  // (MODE_QF) and forms Hess[delta] only for agents that turn out to take a CG step
  bool predict_boundary = true;
  std::vector<double> h_sums;
  // per-iteration trace (dpgo_hip_set_trace): [K][trace_cap][kTraceWidth] doubles
  dpgo::DevBuf<double> trace;
  int trace_cap = 0;
  // in-step SpMM timing (dpgo_rbcd_set_kernel_timing): HIP events around every X.Q launch on the
  // handle's stream, resolved per mode by take_spmm_times()
  int timing = 0;  // 0 off, k > 0: every k-th launch of each mode (a sample: events cost dispatch gaps)
  long long timing_seq[dpgo::kSpmmModes] = {};
  struct TimedLaunch {
    int mode;
    hipEvent_t a, b;
    double frac;  // the launch's tiles / the batch's tiles (a half-batch launch of the split merged tCG: ~0.5)
  };
  std::vector<TimedLaunch> timed;
  std::vector<hipEvent_t> ev_pool;
  // completed timed launches drained out of `timed` (bounded event count on long timed runs)
  double timed_ms[dpgo::kSpmmModes] = {};
  long long timed_n[dpgo::kSpmmModes] = {};
  double timed_frac[dpgo::kSpmmModes] = {};  // summed TimedLaunch::frac: full-batch launch equivalents
  hipEvent_t fac_ev[2] = {nullptr, nullptr};  // the device factorisation's timing (created once per handle)
  ~dpgo_hip_problem_s() {
    for (auto e : fac_ev)
      if (e) (void)hipEventDestroy(e);
    for (auto& t : timed) {
      (void)hipEventDestroy(t.a);
      (void)hipEventDestroy(t.b);
    }
    for (auto e : ev_pool) (void)hipEventDestroy(e);
  }

  size_t vec_len() const { return static_cast<size_t>(N) * r * b; }
  size_t vec_bytes() const { return vec_len() * sizeof(double); }
  size_t s_len() const { return static_cast<size_t>(N) * (b - 1) * b / 2; }  // packed symmetric S per pose
};


namespace dpgo {
// helpers implemented in capi.cpp
LaunchCtx make_ctx(dpgo_hip_problem h, int flag_kind, double* partials);
int problem_ready(dpgo_hip_problem h);
int ensure_work_public(dpgo_hip_problem h);

// PGOAgent status after an update (src/PGOAgent.cpp:700-716): relativeChange of X_out against ref
// (XPrev), readyToTerminate with the converged loop-closure ratio per agent (nullptr = 1).
struct StatusArgs {
  const double* ref;
  const double* conv_ratio;
  double rel_tol, min_ratio;
};
// dpgo_hip_optimize_dev + the status pass (st may be null)
int optimize_dev_status(dpgo_hip_problem h, const dpgo_opt_params* params, const double* X_in, double* X_out,
                        const int* agent_enabled_host, dpgo_opt_result* results, const StatusArgs* st);
// f / |grad|^2 / <G, X> per agent at X into the handle's sums (OP_SUM, nq 3): asynchronous
bool merged_split(dpgo_hip_problem h);  // TUNE_SPLIT_STREAMS applies to this batch (capi.cpp)
int eval_sums_dev(dpgo_hip_problem h, const double* X);
// the same with the edge-stream Q at unit weights (keep_unit_q: the copy taken before any reweighting)
int eval_sums_unit_dev(dpgo_hip_problem h, const double* X);
int keep_unit_q(dpgo_hip_problem h);
// copy the per-agent sums (4 per agent) to the host (synchronises)
int download_sums_public(dpgo_hip_problem h, std::vector<double>& out);
// X.Q launch with the handle's optional event timing
int spmm_launch(dpgo_hip_problem h, int mode, const LaunchCtx& c, const SpmmArgs& a);
// synchronise and add the elapsed ms / launch counts of the timed launches per SpmmMode (kSpmmModes)
int take_spmm_times(dpgo_hip_problem h, double* ms_per_mode, long long* launches_per_mode, double* batch_equiv);
// fold completed (wait: all) timed launches into the handle's per-mode running totals
int drain_timed(dpgo_hip_problem h, bool wait);
}  // namespace dpgo

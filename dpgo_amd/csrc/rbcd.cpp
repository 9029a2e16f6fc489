// Multi-agent RBCD round engine (include/dpgo_rbcd.h).
//
// Mirrors, per agent, PGOAgent::iterate (src/PGOAgent.cpp:642-718) with updateX (:1093-1165),
// constructQMatrix (:720-781), constructGMatrix (:783-859) and the Nesterov updates (:1033-1091),
// under a colour-class schedule: in iteration t the agents of colour c_t are selected
// (doOptimization = true) and every other agent runs iterate(false).  All selected agents of a
// colour that live on this GPU are ONE batched dpgo_hip_problem.  Public poses move between
// ranks through caller-owned device buffers; same-rank neighbours are read in place.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <set>
#include <vector>

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <mutex>
#include <string>

#include "graph_internal.h"

using namespace dpgo;

struct dpgo_rbcd_s {
  int d = 0, r = 0, b = 0, rank = 0, world = 1, K = 0, ncolors = 0;
  dpgo_rbcd_params P;
  std::vector<int> color;                 // per global agent
  std::vector<int> owned;                 // owned global agents, colour-major
  std::vector<int> color_off;             // [ncolors + 1] into owned
  // dpgo_rbcd_set_selected: per owned agent (colour-major, as `owned`) 1 = optimise when its colour is updated;
  // empty = every agent of the colour (the colour schedule)
  std::vector<int> sel_mask;
  DevBuf<int> sel_mask_dev;  // sel_mask on the device (the neighbour-pose snapshot of the selected agents)
  std::vector<long> own_pose_off;         // [owned + 1] pose offsets into owned buffers
  long Nown = 0;
  std::vector<int> own_global;            // owned buffer pose index -> global pose id
  hipStream_t stream = nullptr;           // launch stream (the caller's after dpgo_rbcd_set_stream)
  hipStream_t own_stream = nullptr;       // created and destroyed by the engine
  // N > 1: the selected colour's updateY runs on a side stream while the launch stream does the other
  // colours' iterate(false) and the halo; dpgo_rbcd_update joins it (ev_sel) before its first launch
  hipStream_t side = nullptr;
  hipEvent_t ev_start = nullptr, ev_sel = nullptr;
  bool sel_pending = false;
  int last_color = -1;  // colour of the last pre_exchange (-1 after set_X)
  std::vector<dpgo_hip_problem> prob;     // per colour (nullptr if none owned)
  DevBuf<double> X, Y, V, Xprev;
  // exchange: the public poses' X only.  With Nesterov a receiver uses its neighbours' aux poses
  // (constructGMatrix(neighborAuxPoseDict)), but those neighbours ran iterate(false) this iteration,
  // so their Y equals their X: one copy serves both dictionaries.
  std::vector<long long> send_counts, recv_counts, send_off, recv_off;  // doubles
  long n_send_items = 0, n_recv_poses = 0;
  DevBuf<int> pack_idx, unpack_x;
  // per-colour halo (examples/MultiRobotExample.cpp:188-213 moves only what the selected robot reads): the
  // poses the selected colour's agents read, peer-major, ascending; received poses scatter to their RX slots
  struct Halo {
    std::vector<long long> send_counts, recv_counts, send_off, recv_off;  // doubles
    long n_send = 0, n_recv = 0;
    DevBuf<int> pack_idx, unpack_slot;
  };
  std::vector<Halo*> halo;
  DevBuf<double> RX;   // received neighbour poses used by updates and reweighting
  DevBuf<double> RXc;  // received neighbour poses of a central evaluation (kept apart from RX)
  // status (PGOAgent::iterate, src/PGOAgent.cpp:700-716): per colour, each agent's loop closures (problem
  // edge indices) and converged ratio (GNC_TLS only; otherwise 1)
  struct LcList {
    DevBuf<int> off, idx;
    DevBuf<double> ratio;
    bool valid = false;
  };
  std::vector<LcList*> lc;
  // algorithmic-byte model inputs per colour per agent (dpgo_rbcd_bytes)
  struct AgentSize {
    double n, m_in, m_shared, gslots;
  };
  std::vector<std::vector<AgentSize>> asz;
  double host_bytes = 0.0;  // per-iteration passes counted by the host (combination, G, exchange)
  std::vector<long long> g_store_calls;  // per colour: optimize calls that stored grad(x1)
  // in-step SpMM timing (dpgo_rbcd_set_kernel_timing)
  double spmm_ms[kSpmmModes] = {};
  long long spmm_launches[kSpmmModes] = {};
  // per colour G assembly tables
  struct GTab {
    DevBuf<int> slot_off, src, outgoing;
    DevBuf<double> R, t, kappa, tau, w;
    int nslots = 0;
    long nent = 0;  // shared-edge entries
  };
  std::vector<GTab*> gt;
  // robust cost: per colour, the loop closures its agents reweight and the colour problem's weights
  struct Gnc {
    DevBuf<int> prob_edge, g_entry, src1, src2, agent, nbr_end, dict_ok;
    DevBuf<double> R, t, kappa, tau, w_prob, dict;  // dict: the agents' neighborPoseDict entries (GncEntries)
    int n = 0;
  };
  std::vector<Gnc*> gnc;
  double mu = 0.0;       // RobustCost::mu (every agent updates it at the same iterations)
  int gnc_iter = 0;      // RobustCost::mGNCIteration
  bool gnc_due = false;  // this iteration reweights (set in pre_exchange, used by update)
  double gamma = 0.0, alpha = 0.0;
  // per colour: the selected agents' updateV (src/PGOAgent.cpp:1086-1091) is deferred into that
  // colour's next combination pass (k_polar_vnext) with the gamma it was due with
  std::vector<char> v_pending;
  std::vector<double> v_gamma;
  long iteration = 0;
  long long agent_updates = 0;
  // native exchange (dpgo_rbcd_comm_init / dpgo_rbcd_exchange): RCCL communicator over the ranks and
  // engine-owned send / receive buffers in the all_to_all layout (peer-major, send_off / recv_off)
  ncclComm_t comm = nullptr;
  bool own_comm = false;
  DevBuf<double> xsend, xrecv;

  ~dpgo_rbcd_s();
  void release() {
    for (auto* p : prob)
      if (p) dpgo_hip_problem_destroy(p);
    for (auto* g : gt) delete g;
    for (auto* g : gnc) delete g;
    for (auto* l : lc) delete l;
    for (auto* x : halo) delete x;
  }
  size_t rb() const { return static_cast<size_t>(r) * b; }
};

namespace {

template <typename T>
int upload_vec(DevBuf<T>& dst, const std::vector<T>& src, hipStream_t s) {
  HIP_TRY(dst.ensure(std::max<size_t>(src.size(), 1)));
  if (!src.empty()) HIP_TRY(hipMemcpyAsync(dst.p, src.data(), sizeof(T) * src.size(), hipMemcpyHostToDevice, s));
  return DPGO_HIP_OK;
}

double* color_ptr(dpgo_rbcd e, DevBuf<double>& buf, int c) {
  return buf.p + static_cast<size_t>(e->own_pose_off[e->color_off[c]]) * e->rb();
}

long color_first_pose(dpgo_rbcd e, int c) { return e->own_pose_off[e->color_off[c]]; }
long color_num_poses(dpgo_rbcd e, int c) { return e->own_pose_off[e->color_off[c + 1]] - e->own_pose_off[e->color_off[c]]; }
double pose_bytes(dpgo_rbcd e) { return 8.0 * static_cast<double>(e->rb()); }

int polar(dpgo_rbcd e, int c, const double* A, const double* B, double ca, double cb, double* out,
          const double* C = nullptr, double* out2 = nullptr, double* xcopy = nullptr, hipStream_t on = nullptr) {
  dpgo_hip_problem h = e->prob[c];
  if (!h) return DPGO_HIP_OK;
  // uniform Nesterov coefficients travel as kernel arguments
  auto ctx = make_ctx(h, FLAG_NONE, h->pa.p);
  if (on) ctx.stream = on;
  HIP_TRY(launch_polar_comb(e->r, e->b, ctx, A, B, nullptr, nullptr, out, C, ca, cb, out2, xcopy));
  e->host_bytes += pose_bytes(e) * static_cast<double>(color_num_poses(e, c)) *
                   (1.0 + (B ? 1.0 : 0.0) + (C ? 1.0 : 0.0) + 1.0 + (out2 ? 1.0 : 0.0) + (xcopy ? 1.0 : 0.0));
  return DPGO_HIP_OK;
}

// out = project((1 - alpha) X + alpha V) for colour c, preceded by the colour's deferred updateV
// V = project(V + gamma (X - Y)) in the same pass when one is pending.  xcopy: XPrev = X (the selected
// colour's status reference) written from the same loads.
int nesterov_comb(dpgo_rbcd e, int c, double* out, double* xcopy = nullptr, hipStream_t on = nullptr) {
  dpgo_hip_problem h = e->prob[c];
  if (!h) return DPGO_HIP_OK;
  double* Xc = color_ptr(e, e->X, c);
  double* Yc = color_ptr(e, e->Y, c);
  double* Vc = color_ptr(e, e->V, c);
  if (!e->v_pending[c]) return polar(e, c, Xc, Vc, 1.0 - e->alpha, e->alpha, out, nullptr, nullptr, xcopy, on);
  e->v_pending[c] = 0;
  auto ctx = make_ctx(h, FLAG_NONE, h->pa.p);
  if (on) ctx.stream = on;
  HIP_TRY(launch_polar_vnext(e->r, e->b, ctx, Xc, Vc, Yc, e->v_gamma[c], 1.0 - e->alpha, e->alpha, out, xcopy));
  e->host_bytes += pose_bytes(e) * static_cast<double>(color_num_poses(e, c)) * (5.0 + (xcopy ? 1.0 : 0.0));
  return DPGO_HIP_OK;
}

int copy_poses(dpgo_rbcd e, double* dst, const double* src, long first_pose, long count) {
  if (count <= 0) return DPGO_HIP_OK;
  HIP_TRY(hipMemcpyAsync(dst + first_pose * e->rb(), src + first_pose * e->rb(), sizeof(double) * count * e->rb(),
                         hipMemcpyDeviceToDevice, e->stream));
  e->host_bytes += 2.0 * pose_bytes(e) * static_cast<double>(count);
  return DPGO_HIP_OK;
}

// constructGMatrix (src/PGOAgent.cpp:783-859) for colour c from in-place neighbours (X) and received
// ones (Rx).  In-place neighbours are never in colour c, so they ran iterate(false) this iteration
// and their aux pose equals X (see dpgo_rbcd_pre_exchange): X serves both dictionaries.
int assemble_G(dpgo_rbcd e, int c, const double* Rx, bool unit_weights = false) {
  dpgo_hip_problem h = e->prob[c];
  if (!h || e->gt[c]->nslots == 0) return DPGO_HIP_OK;
  auto* t = e->gt[c];
  GEdges ge{t->slot_off.p, t->src.p, t->outgoing.p, t->R.p, t->t.p, t->kappa.p, t->tau.p,
            unit_weights ? nullptr : t->w.p};
  HIP_TRY(launch_assemble_G(e->r, e->b, ge, t->nslots, e->X.p, Rx, h->gblk.p, e->stream));
  // per entry: neighbour pose + measurement (R, t, kappa, tau, w, src, outgoing); per slot: G block
  const double d = e->d;
  e->host_bytes += static_cast<double>(t->nent) * (pose_bytes(e) + 8.0 * (d * d + d + 3.0) + 8.0) +
                   static_cast<double>(t->nslots) * (pose_bytes(e) + 4.0);
  return DPGO_HIP_OK;
}

// GNC / robust reweighting of colour c's loop closures at the current poses (own X buffer and the
// received neighbour poses), then the on-device rebuild of the colour problem's Q.
int reweight_color(dpgo_rbcd e, int c) {
  dpgo_hip_problem h = e->prob[c];
  if (!h) return DPGO_HIP_OK;
  auto* g = e->gnc[c];
  const GncEntries ge{g->n, g->prob_edge.p, g->g_entry.p, g->src1.p, g->src2.p, g->R.p, g->t.p, g->kappa.p,
                      g->tau.p, g->agent.p, g->nbr_end.p, g->dict.p, g->dict_ok.p};
  const RobustParams rp{e->P.robust_cost, e->mu, e->P.gnc_barc, e->P.huber_threshold, e->P.tls_threshold};
  HIP_TRY(launch_gnc_weights(e->r, e->b, ge, e->X.p, e->RX.p, rp, g->w_prob.p, e->gt[c]->w.p, e->stream));
  DPGO_TRY(dpgo_hip_set_edge_weights_dev(h, g->w_prob.p));
  if (e->P.robust_cost == DPGO_ROBUST_GNC_TLS) {  // computeConvergedLoopClosureRatio (:1247-1289)
    auto* l = e->lc[c];
    HIP_TRY(launch_conv_ratio(h->K, l->off.p, l->idx.p, g->w_prob.p, l->ratio.p, e->stream));
    l->valid = true;
  }
  return DPGO_HIP_OK;
}

// updateNeighborPoses for the selected agents of colour c (examples/MultiRobotExample.cpp:188-213): each shared loop
// closure they reweight records the neighbour pose they now hold (this iteration's halo / same-rank X), which their
// updateLoopClosuresWeights reads at any later reweighting (src/PGOAgent.cpp:1201-1235), whichever colour order
// and whichever rank count: no reweighting reads a received pose older than the agent's own last selection.
int snapshot_neighbors(dpgo_rbcd e, int c) {
  auto* g = e->gnc[c];
  if (!e->prob[c] || g->n == 0) return DPGO_HIP_OK;
  const GncEntries ge{g->n, g->prob_edge.p, g->g_entry.p, g->src1.p, g->src2.p, g->R.p, g->t.p, g->kappa.p,
                      g->tau.p, g->agent.p, g->nbr_end.p, g->dict.p, g->dict_ok.p};
  const int* mask = e->sel_mask.empty() ? nullptr : e->sel_mask_dev.p + e->color_off[c];
  HIP_TRY(launch_gnc_snapshot(e->r, e->b, ge, e->X.p, e->RX.p, mask, e->stream));
  return DPGO_HIP_OK;
}

// QuadraticOptimizer as PGOAgent::updateX configures it (src/PGOAgent.cpp:1131-1137), plus the agent
// status against status_ref (XPrev) when the engine tracks it.
int optimize_color(dpgo_rbcd e, int c, const double* Xin, double* Xout, dpgo_opt_result* results,
                   const double* status_ref) {
  dpgo_hip_problem h = e->prob[c];
  if (!h) return DPGO_HIP_OK;
  dpgo_opt_params p;
  dpgo_hip_default_params(&p);
  p.algorithm = e->P.algorithm;
  p.tr_iterations = 1;
  p.tr_tolerance = e->P.tolerance;
  p.tr_max_inner = e->P.max_inner;
  p.tr_initial_radius = e->P.initial_radius;
  p.precon = e->P.precon;
  StatusArgs st{status_ref, e->lc[c]->valid ? e->lc[c]->ratio.p : nullptr, e->P.rel_change_tol,
                e->P.min_convergence_ratio};
  if (!h->predict_boundary) e->g_store_calls[c] += 1;  // EVAL_TCG stores grad(x1) (byte model)
  // a selection inside the colour (the example's greedy robot, dpgo_rbcd_set_selected): the others keep X_in, which
  // is PGOAgent::updateX(false) -- X = Y with acceleration, X unchanged without
  const int* en = e->sel_mask.empty() ? nullptr : e->sel_mask.data() + e->color_off[c];
  DPGO_TRY(optimize_dev_status(h, &p, Xin, Xout, en, results, status_ref ? &st : nullptr));
  int n_up = h->K;
  if (en) n_up = static_cast<int>(std::count(en, en + h->K, 1));
  e->agent_updates += n_up;
  return DPGO_HIP_OK;
}

// Public poses this rank must send to / receive from every peer: endpoints of edges that join
// agents on different ranks, in ascending global pose id (identical on every rank).
void exchange_plan(dpgo_graph g, const int* agent_of_pose, const int* agent_rank, int rank, int world,
                   std::vector<std::set<int>>& send_set, std::vector<std::set<int>>& recv_set) {
  send_set.assign(world, {});
  recv_set.assign(world, {});
  for (size_t k = 0; k < g->p1.size(); ++k) {
    const int i = g->p1[k], j = g->p2[k];
    const int ri = agent_rank[agent_of_pose[i]], rj = agent_rank[agent_of_pose[j]];
    if (agent_of_pose[i] == agent_of_pose[j] || ri == rj) continue;
    if (ri == rank) {
      send_set[rj].insert(i);
      recv_set[rj].insert(j);
    } else if (rj == rank) {
      send_set[ri].insert(j);
      recv_set[ri].insert(i);
    }
  }
}

// The public poses the agents of colour c read this iteration: pose i (owned here) goes to peer q when an
// edge joins it to a pose of q whose agent has colour c; pose j of peer q comes here when it joins an owned
// pose whose agent has colour c.
void exchange_plan_color(dpgo_graph g, const int* agent_of_pose, const int* agent_rank, const std::vector<int>& color,
                         int c, int rank, int world, std::vector<std::set<int>>& send_set,
                         std::vector<std::set<int>>& recv_set) {
  send_set.assign(world, {});
  recv_set.assign(world, {});
  for (size_t k = 0; k < g->p1.size(); ++k) {
    const int i = g->p1[k], j = g->p2[k];
    const int ai = agent_of_pose[i], aj = agent_of_pose[j];
    const int ri = agent_rank[ai], rj = agent_rank[aj];
    if (ai == aj || ri == rj) continue;
    if (ri == rank) {
      if (color[aj] == c) send_set[rj].insert(i);
      if (color[ai] == c) recv_set[rj].insert(j);
    } else if (rj == rank) {
      if (color[ai] == c) send_set[ri].insert(j);
      if (color[aj] == c) recv_set[ri].insert(i);
    }
  }
}

// greedy colouring of the agent-adjacency graph in agent-id order (every rank computes the same)
int agent_colors(dpgo_graph g, int num_agents, const int* agent_of_pose, std::vector<int>& color) {
  std::vector<std::set<int>> adj(num_agents);
  for (size_t k = 0; k < g->p1.size(); ++k) {
    const int a1 = agent_of_pose[g->p1[k]], a2 = agent_of_pose[g->p2[k]];
    if (a1 != a2) {
      adj[a1].insert(a2);
      adj[a2].insert(a1);
    }
  }
  color.assign(num_agents, -1);
  int ncolors = 0;
  for (int a = 0; a < num_agents; ++a) {
    std::set<int> used;
    for (int nb : adj[a])
      if (color[nb] >= 0) used.insert(color[nb]);
    int c = 0;
    while (used.count(c)) ++c;
    color[a] = c;
    ncolors = std::max(ncolors, c + 1);
  }
  return ncolors;
}

}  // namespace

extern "C" {

int dpgo_rbcd_plan_color(dpgo_graph g, int num_agents, const int* agent_of_pose, const int* agent_rank, int color,
                         int rank, int world, long long* send_counts, long long* recv_counts, int* send_poses,
                         int* recv_poses) {
  if (!g || !agent_of_pose || !agent_rank || world <= 0 || rank < 0 || rank >= world || num_agents <= 0)
    return fail(DPGO_HIP_EINVAL, "bad plan arguments");
  for (int i = 0; i < g->n; ++i)
    if (agent_of_pose[i] < 0 || agent_of_pose[i] >= num_agents) return fail(DPGO_HIP_EINVAL, "agent_of_pose out of range");
  std::vector<int> col;
  const int nc = agent_colors(g, num_agents, agent_of_pose, col);
  if (color < 0 || color >= nc) return fail(DPGO_HIP_EINVAL, "bad colour");
  std::vector<std::set<int>> ss, rs;
  exchange_plan_color(g, agent_of_pose, agent_rank, col, color, rank, world, ss, rs);
  long long so = 0, ro = 0;
  for (int p = 0; p < world; ++p) {
    if (send_counts) send_counts[p] = static_cast<long long>(ss[p].size());
    if (recv_counts) recv_counts[p] = static_cast<long long>(rs[p].size());
    if (send_poses)
      for (int x : ss[p]) send_poses[so++] = x;
    if (recv_poses)
      for (int x : rs[p]) recv_poses[ro++] = x;
  }
  return DPGO_HIP_OK;
}

int dpgo_rbcd_plan(dpgo_graph g, int num_agents, const int* agent_of_pose, const int* agent_rank, int rank, int world,
                   long long* send_counts, long long* recv_counts, int* send_poses, int* recv_poses) {
  if (!g || !agent_of_pose || !agent_rank || world <= 0 || rank < 0 || rank >= world || num_agents <= 0)
    return fail(DPGO_HIP_EINVAL, "bad plan arguments");
  for (int i = 0; i < g->n; ++i)
    if (agent_of_pose[i] < 0 || agent_of_pose[i] >= num_agents) return fail(DPGO_HIP_EINVAL, "agent_of_pose out of range");
  std::vector<std::set<int>> ss, rs;
  exchange_plan(g, agent_of_pose, agent_rank, rank, world, ss, rs);
  long long so = 0, ro = 0;
  for (int p = 0; p < world; ++p) {
    if (send_counts) send_counts[p] = static_cast<long long>(ss[p].size());
    if (recv_counts) recv_counts[p] = static_cast<long long>(rs[p].size());
    if (send_poses)
      for (int x : ss[p]) send_poses[so++] = x;
    if (recv_poses)
      for (int x : rs[p]) recv_poses[ro++] = x;
  }
  return DPGO_HIP_OK;
}

void dpgo_rbcd_default_params(dpgo_rbcd_params* p) {
  if (!p) return;
  p->r = 5;
  p->acceleration = 0;
  p->restart_interval = 30;
  p->max_inner = 10;
  p->initial_radius = 100.0;
  p->tolerance = 1e-2;
  p->precon = DPGO_PRECON_BLOCK_JACOBI;
  p->algorithm = DPGO_ALG_RTR;
  p->q_format = DPGO_QFMT_EDGES;
  p->robust_cost = DPGO_ROBUST_L2;
  p->robust_opt_inner_iters = 30;
  p->gnc_max_iters = 100;
  p->gnc_barc = 10.0;
  p->gnc_mu_step = 1.4;
  p->gnc_init_mu = 1e-4;
  p->huber_threshold = 3.0;
  p->tls_threshold = 10.0;
  p->status = 1;
  p->rel_change_tol = 5e-3;
  p->min_convergence_ratio = 0.8;
}

int dpgo_rbcd_create(dpgo_graph g, int num_agents, const int* agent_of_pose, const int* agent_rank, int rank,
                     int world, const dpgo_rbcd_params* params, dpgo_rbcd* out) {
  if (!g || !agent_of_pose || !agent_rank || !out || num_agents <= 0 || world <= 0 || rank < 0 || rank >= world)
    return fail(DPGO_HIP_EINVAL, "bad rbcd arguments");
  *out = nullptr;
  if (usable_devices() == 0) return fail(DPGO_HIP_ENODEV, "no gfx950 device available (no CPU fallback)");
  auto* e = new dpgo_rbcd_s();
  auto bail = [&](int rc) {
    delete e;
    return rc;
  };
  if (params)
    e->P = *params;
  else
    dpgo_rbcd_default_params(&e->P);
  if (e->P.robust_cost != DPGO_ROBUST_L2 && e->P.q_format != DPGO_QFMT_EDGES)
    return bail(fail(DPGO_HIP_EINVAL, "robust costs reweight an edge-stream Q (q_format DPGO_QFMT_EDGES)"));
  if (e->P.robust_cost < DPGO_ROBUST_L2 || e->P.robust_cost > DPGO_ROBUST_GNC_TLS || e->P.robust_opt_inner_iters <= 0)
    return bail(fail(DPGO_HIP_EINVAL, "bad robust cost parameters"));
  e->mu = e->P.gnc_init_mu;  // RobustCost::reset (src/DPGO_robust.cpp:70-84)
  e->d = g->d;
  e->r = e->P.r;
  e->b = g->d + 1;
  e->rank = rank;
  e->world = world;
  e->K = num_agents;
  const int n = g->n, d = g->d;
  const size_t m = g->p1.size();
  // local index of every pose inside its agent (global order)
  std::vector<int> local(n), agent_n(num_agents, 0);
  for (int i = 0; i < n; ++i) {
    const int a = agent_of_pose[i];
    if (a < 0 || a >= num_agents) return bail(fail(DPGO_HIP_EINVAL, "agent_of_pose out of range"));
    local[i] = agent_n[a]++;
  }
  for (int a = 0; a < num_agents; ++a)
    if (agent_n[a] == 0) return bail(fail(DPGO_HIP_EINVAL, "every agent needs >= 1 pose"));
  // greedy colouring of the agent adjacency in agent-id order
  e->ncolors = agent_colors(g, num_agents, agent_of_pose, e->color);
  // owned agents, colour-major
  e->color_off.assign(e->ncolors + 1, 0);
  for (int c = 0; c < e->ncolors; ++c) {
    for (int a = 0; a < num_agents; ++a)
      if (agent_rank[a] == rank && e->color[a] == c) e->owned.push_back(a);
    e->color_off[c + 1] = static_cast<int>(e->owned.size());
  }
  std::vector<int> owned_pos(num_agents, -1);
  e->own_pose_off.assign(e->owned.size() + 1, 0);
  for (size_t q = 0; q < e->owned.size(); ++q) {
    owned_pos[e->owned[q]] = static_cast<int>(q);
    e->own_pose_off[q + 1] = e->own_pose_off[q] + agent_n[e->owned[q]];
  }
  e->Nown = e->own_pose_off.back();
  e->own_global.assign(e->Nown, -1);
  for (int i = 0; i < n; ++i) {
    const int q = owned_pos[agent_of_pose[i]];
    if (q >= 0) e->own_global[e->own_pose_off[q] + local[i]] = i;
  }
  auto owned_index = [&](int pose) -> long {
    const int q = owned_pos[agent_of_pose[pose]];
    return q < 0 ? -1 : e->own_pose_off[q] + local[pose];
  };
  // ---- exchange plan: poses each peer needs from us / we need from each peer (sorted global ids)
  std::vector<std::set<int>> send_set, recv_set;
  exchange_plan(g, agent_of_pose, agent_rank, rank, world, send_set, recv_set);
  const long long rbd = static_cast<long long>(e->rb());
  e->send_counts.assign(world, 0);
  e->recv_counts.assign(world, 0);
  e->send_off.assign(world + 1, 0);
  e->recv_off.assign(world + 1, 0);
  std::vector<int> pack_idx, unpack_x;
  std::map<int, long> recv_slot;  // global pose -> recv pose index
  long rs = 0;
  for (int p = 0; p < world; ++p) {
    const long cnt_s = static_cast<long>(send_set[p].size()), cnt_r = static_cast<long>(recv_set[p].size());
    e->send_counts[p] = cnt_s * rbd;
    e->recv_counts[p] = cnt_r * rbd;
    e->send_off[p + 1] = e->send_off[p] + e->send_counts[p];
    e->recv_off[p + 1] = e->recv_off[p] + e->recv_counts[p];
    for (int pose : send_set[p]) pack_idx.push_back(static_cast<int>(owned_index(pose)));
    const long base = e->recv_off[p] / rbd;  // recv segment start in poses
    long s = 0;
    for (int pose : recv_set[p]) {
      recv_slot[pose] = rs++;
      unpack_x.push_back(static_cast<int>(base + s));
      ++s;
    }
  }
  e->n_send_items = static_cast<long>(pack_idx.size());
  e->n_recv_poses = rs;
  // per-colour plans over the same RX slots
  e->halo.assign(e->ncolors, nullptr);
  std::vector<std::vector<int>> halo_pack(e->ncolors), halo_unpack(e->ncolors);
  for (int c = 0; c < e->ncolors; ++c) {
    auto* H = e->halo[c] = new dpgo_rbcd_s::Halo();
    std::vector<std::set<int>> ss, rr;
    exchange_plan_color(g, agent_of_pose, agent_rank, e->color, c, rank, world, ss, rr);
    H->send_counts.assign(world, 0);
    H->recv_counts.assign(world, 0);
    H->send_off.assign(world + 1, 0);
    H->recv_off.assign(world + 1, 0);
    for (int p = 0; p < world; ++p) {
      H->send_counts[p] = static_cast<long long>(ss[p].size()) * rbd;
      H->recv_counts[p] = static_cast<long long>(rr[p].size()) * rbd;
      H->send_off[p + 1] = H->send_off[p] + H->send_counts[p];
      H->recv_off[p + 1] = H->recv_off[p] + H->recv_counts[p];
      for (int pose : ss[p]) halo_pack[c].push_back(static_cast<int>(owned_index(pose)));
      for (int pose : rr[p]) halo_unpack[c].push_back(static_cast<int>(recv_slot.at(pose)));
    }
    H->n_send = static_cast<long>(halo_pack[c].size());
    H->n_recv = static_cast<long>(halo_unpack[c].size());
  }
  if (hipStreamCreateWithFlags(&e->own_stream, hipStreamNonBlocking) != hipSuccess)
    return bail(fail(DPGO_HIP_EDEVICE, "stream create failed"));
  e->stream = e->own_stream;
  if (world > 1 && (hipStreamCreateWithFlags(&e->side, hipStreamNonBlocking) != hipSuccess ||
                    hipEventCreateWithFlags(&e->ev_start, hipEventDisableTiming) != hipSuccess ||
                    hipEventCreateWithFlags(&e->ev_sel, hipEventDisableTiming) != hipSuccess))
    return bail(fail(DPGO_HIP_EDEVICE, "side stream create failed"));
  int rc = upload_vec(e->pack_idx, pack_idx, e->stream);
  if (rc == DPGO_HIP_OK) rc = upload_vec(e->unpack_x, unpack_x, e->stream);
  for (int c = 0; c < e->ncolors && rc == DPGO_HIP_OK; ++c) {
    rc = upload_vec(e->halo[c]->pack_idx, halo_pack[c], e->stream);
    if (rc == DPGO_HIP_OK) rc = upload_vec(e->halo[c]->unpack_slot, halo_unpack[c], e->stream);
  }
  if (rc != DPGO_HIP_OK) return bail(rc);
  if (e->RX.ensure(std::max<long>(rs, 1) * e->rb()) != hipSuccess || e->RXc.ensure(std::max<long>(rs, 1) * e->rb()) != hipSuccess ||
      e->X.ensure(std::max<long>(e->Nown, 1) * e->rb()) != hipSuccess ||
      e->Y.ensure(std::max<long>(e->Nown, 1) * e->rb()) != hipSuccess ||
      e->V.ensure(std::max<long>(e->Nown, 1) * e->rb()) != hipSuccess ||
      e->Xprev.ensure(std::max<long>(e->Nown, 1) * e->rb()) != hipSuccess)
    return bail(fail(DPGO_HIP_ENOMEM, "device allocation failed"));
  e->v_pending.assign(e->ncolors, 0);
  e->v_gamma.assign(e->ncolors, 0.0);

  // ---- per owned agent: Q (private edges + shared-edge diagonal terms) and shared edges
  std::vector<std::vector<size_t>> agent_edges(e->owned.size());
  for (size_t k = 0; k < m; ++k) {
    const int q1 = owned_pos[agent_of_pose[g->p1[k]]], q2 = owned_pos[agent_of_pose[g->p2[k]]];
    if (q1 >= 0) agent_edges[q1].push_back(k);
    if (q2 >= 0 && q2 != q1) agent_edges[q2].push_back(k);
  }
  e->prob.assign(e->ncolors, nullptr);
  e->gt.assign(e->ncolors, nullptr);
  e->gnc.assign(e->ncolors, nullptr);
  e->lc.assign(e->ncolors, nullptr);
  e->asz.assign(e->ncolors, {});
  e->g_store_calls.assign(e->ncolors, 0);
  for (int c = 0; c < e->ncolors; ++c) {
    e->gt[c] = new dpgo_rbcd_s::GTab();
    e->gnc[c] = new dpgo_rbcd_s::Gnc();
    e->lc[c] = new dpgo_rbcd_s::LcList();
    std::vector<int> lc_off{0}, lc_idx;  // every loop closure of each agent (converged ratio)
    const int a0 = e->color_off[c], a1 = e->color_off[c + 1];
    // loop closures this colour reweights (PGOAgent::updateLoopClosuresWeights): private ones that
    // are not odometry (local p2 != p1 + 1, as the partition's split), and shared ones whose other
    // agent has the larger ID (only the lower-ID agent updates its copy)
    std::vector<int> gn_pe, gn_ge, gn_s1, gn_s2, gn_agent, gn_nbr;
    std::vector<double> gn_R, gn_t, gn_k, gn_tau;
    long prob_edges = 0;
    if (a1 == a0) continue;
    std::vector<int> counts;
    for (int q = a0; q < a1; ++q) counts.push_back(agent_n[e->owned[q]]);
    dpgo_hip_problem h = nullptr;
    rc = dpgo_hip_problem_create_batch(a1 - a0, counts.data(), d, e->r, &h);
    if (rc != DPGO_HIP_OK) return bail(rc);
    e->prob[c] = h;
    h->stream = e->stream;
    std::vector<int> slot_off{0}, src, outgoing;
    std::vector<double> Rv, tv, kv, tauv, wv;
    for (int q = a0; q < a1; ++q) {
      const int A = e->owned[q];
      // Q_A as its measurement stream: private edges with both local endpoints, shared edges with
      // the foreign endpoint set to -1 (diagonal terms only, :754-760 / :770-775)
      std::map<int, std::vector<size_t>> slots;  // local public pose -> shared edges
      std::vector<int> ep1, ep2;
      std::vector<double> eR, et, ek, etau;
      for (size_t k : agent_edges[q]) {
        const int i = g->p1[k], j = g->p2[k];
        const bool own_i = agent_of_pose[i] == A, own_j = agent_of_pose[j] == A;
        ep1.push_back(own_i ? local[i] : -1);
        ep2.push_back(own_j ? local[j] : -1);
        eR.insert(eR.end(), &g->R[k * d * d], &g->R[k * d * d] + d * d);
        et.insert(et.end(), &g->t[k * d], &g->t[k * d] + d);
        ek.push_back(g->kappa[k]);
        etau.push_back(g->tau[k]);
        if (!(own_i && own_j)) slots[own_i ? local[i] : local[j]].push_back(k);
      }
      if (e->P.q_format == DPGO_QFMT_BSR) {  // explicit Q_A (BSR), as the reference materialises it
        BsrBuilder B(agent_n[A], e->b);
        for (size_t x = 0; x < ep1.size(); ++x)
          if (ep1[x] >= 0 && ep2[x] >= 0) {
            B.touch(ep1[x], ep2[x]);
            B.touch(ep2[x], ep1[x]);
          }
        B.freeze();
        double Wii[16], Wjj[16], Wij[16], Wji[16];
        for (size_t x = 0; x < ep1.size(); ++x) {
          edge_blocks(d, &eR[x * d * d], &et[x * d], ek[x], etau[x], 1.0, Wii, Wjj, Wij, Wji);
          if (ep1[x] >= 0) B.add(ep1[x], ep1[x], Wii);
          if (ep2[x] >= 0) B.add(ep2[x], ep2[x], Wjj);
          if (ep1[x] >= 0 && ep2[x] >= 0) {
            B.add(ep1[x], ep2[x], Wij);
            B.add(ep2[x], ep1[x], Wji);
          }
        }
        rc = dpgo_hip_set_Q_bsr(h, q - a0, agent_n[A], B.out.rowptr.data(), B.out.col.data(), B.out.blocks.data());
      } else {
        rc = dpgo_hip_set_Q_edges(h, q - a0, static_cast<int>(ep1.size()), ep1.data(), ep2.data(), eR.data(),
                                  et.data(), ek.data(), etau.data(), nullptr);
      }
      if (rc != DPGO_HIP_OK) return bail(rc);
      std::map<size_t, int> g_index;  // shared edge -> its entry in the colour's G table
      std::vector<int> gpose;
      for (auto& kv2 : slots) {
        gpose.push_back(kv2.first);
        for (size_t k : kv2.second) {
          g_index[k] = static_cast<int>(src.size());
          const int i = g->p1[k], j = g->p2[k];
          const bool out_edge = agent_of_pose[i] == A;
          const int nbr = out_edge ? j : i;
          const long oi = owned_index(nbr);
          src.push_back(oi >= 0 ? static_cast<int>(oi) : -1 - static_cast<int>(recv_slot.at(nbr)));
          outgoing.push_back(out_edge ? 1 : 0);
          Rv.insert(Rv.end(), &g->R[k * d * d], &g->R[k * d * d] + d * d);
          tv.insert(tv.end(), &g->t[k * d], &g->t[k * d] + d);
          kv.push_back(g->kappa[k]);
          tauv.push_back(g->tau[k]);
          wv.push_back(1.0);
        }
        slot_off.push_back(static_cast<int>(src.size()));
      }
      dpgo_rbcd_s::AgentSize sz{static_cast<double>(agent_n[A]), 0.0, 0.0, static_cast<double>(gpose.size())};
      for (size_t x = 0; x < agent_edges[q].size(); ++x) {
        const size_t k = agent_edges[q][x];
        const int i = g->p1[k], j = g->p2[k];
        const bool own_i = agent_of_pose[i] == A, own_j = agent_of_pose[j] == A;
        if (own_i && own_j)
          sz.m_in += 1.0;
        else
          sz.m_shared += 1.0;
        // loop closures (odometry = consecutive local indices, as the partition splits them)
        if (!(own_i && own_j && local[j] == local[i] + 1)) lc_idx.push_back(static_cast<int>(prob_edges + static_cast<long>(x)));
      }
      e->asz[c].push_back(sz);
      lc_off.push_back(static_cast<int>(lc_idx.size()));
      for (size_t x = 0; x < agent_edges[q].size(); ++x) {
        const size_t k = agent_edges[q][x];
        const int i = g->p1[k], j = g->p2[k];
        const bool own_i = agent_of_pose[i] == A, own_j = agent_of_pose[j] == A;
        int ge = -1;
        if (own_i && own_j) {
          if (local[j] == local[i] + 1) continue;  // odometry: never reweighted
        } else {
          const int other = own_i ? agent_of_pose[j] : agent_of_pose[i];
          if (other < A) continue;  // the lower-ID agent is responsible (:1201-1235)
          ge = g_index.at(k);
        }
        auto src_of = [&](int pose) -> int {
          const long oi = owned_index(pose);
          return oi >= 0 ? static_cast<int>(oi) : -1 - static_cast<int>(recv_slot.at(pose));
        };
        gn_pe.push_back(static_cast<int>(prob_edges + static_cast<long>(x)));
        gn_ge.push_back(ge);
        gn_agent.push_back(q - a0);
        gn_nbr.push_back(ge < 0 ? -1 : own_i ? 1 : 0);  // a shared edge: the endpoint this agent does not own
        gn_s1.push_back(src_of(i));
        gn_s2.push_back(src_of(j));
        gn_R.insert(gn_R.end(), &g->R[k * d * d], &g->R[k * d * d] + d * d);
        gn_t.insert(gn_t.end(), &g->t[k * d], &g->t[k * d] + d);
        gn_k.push_back(g->kappa[k]);
        gn_tau.push_back(g->tau[k]);
      }
      prob_edges += static_cast<long>(agent_edges[q].size());
      std::vector<double> zeros(gpose.size() * e->rb(), 0.0);
      rc = dpgo_hip_set_G(h, q - a0, static_cast<int>(gpose.size()), gpose.data(), zeros.data());
      if (rc != DPGO_HIP_OK) return bail(rc);
    }
    rc = problem_ready(h);  // uploads Q, block-Jacobi inverses, G slot map
    if (rc == DPGO_HIP_OK && e->P.robust_cost != DPGO_ROBUST_L2) rc = keep_unit_q(h);  // the central evaluation's Q
    if (rc != DPGO_HIP_OK) return bail(rc);
    auto* t = e->gt[c];
    t->nslots = static_cast<int>(slot_off.size()) - 1;
    t->nent = static_cast<long>(src.size());
    {
      auto* l = e->lc[c];
      rc = upload_vec(l->off, lc_off, e->stream);
      if (rc == DPGO_HIP_OK) rc = upload_vec(l->idx, lc_idx, e->stream);
      if (rc == DPGO_HIP_OK && l->ratio.ensure(a1 - a0) != hipSuccess) rc = fail(DPGO_HIP_ENOMEM, "ratio");
      if (rc != DPGO_HIP_OK) return bail(rc);
    }
    if (t->nslots != h->num_gslots) return bail(fail(DPGO_HIP_ESTATE, "G slot order mismatch"));
    rc = upload_vec(t->slot_off, slot_off, e->stream);
    if (rc == DPGO_HIP_OK) rc = upload_vec(t->src, src, e->stream);
    if (rc == DPGO_HIP_OK) rc = upload_vec(t->outgoing, outgoing, e->stream);
    if (rc == DPGO_HIP_OK) rc = upload_vec(t->R, Rv, e->stream);
    if (rc == DPGO_HIP_OK) rc = upload_vec(t->t, tv, e->stream);
    if (rc == DPGO_HIP_OK) rc = upload_vec(t->kappa, kv, e->stream);
    if (rc == DPGO_HIP_OK) rc = upload_vec(t->tau, tauv, e->stream);
    if (rc == DPGO_HIP_OK) rc = upload_vec(t->w, wv, e->stream);
    auto* gc = e->gnc[c];
    gc->n = static_cast<int>(gn_pe.size());
    if (rc == DPGO_HIP_OK) rc = upload_vec(gc->prob_edge, gn_pe, e->stream);
    if (rc == DPGO_HIP_OK) rc = upload_vec(gc->g_entry, gn_ge, e->stream);
    if (rc == DPGO_HIP_OK) rc = upload_vec(gc->src1, gn_s1, e->stream);
    if (rc == DPGO_HIP_OK) rc = upload_vec(gc->src2, gn_s2, e->stream);
    if (rc == DPGO_HIP_OK) rc = upload_vec(gc->R, gn_R, e->stream);
    if (rc == DPGO_HIP_OK) rc = upload_vec(gc->t, gn_t, e->stream);
    if (rc == DPGO_HIP_OK) rc = upload_vec(gc->kappa, gn_k, e->stream);
    if (rc == DPGO_HIP_OK) rc = upload_vec(gc->tau, gn_tau, e->stream);
    if (rc == DPGO_HIP_OK) rc = upload_vec(gc->agent, gn_agent, e->stream);
    if (rc == DPGO_HIP_OK) rc = upload_vec(gc->nbr_end, gn_nbr, e->stream);
    if (rc == DPGO_HIP_OK) rc = upload_vec(gc->dict_ok, std::vector<int>(std::max<size_t>(gn_pe.size(), 1), 0), e->stream);
    if (rc == DPGO_HIP_OK && gc->dict.ensure(std::max<size_t>(gn_pe.size(), 1) * e->rb()) != hipSuccess)
      rc = fail(DPGO_HIP_ENOMEM, "GNC neighbour dictionary");
    if (rc == DPGO_HIP_OK) rc = upload_vec(gc->w_prob, std::vector<double>(std::max<long>(prob_edges, 1), 1.0), e->stream);
    if (rc == DPGO_HIP_OK && hipStreamSynchronize(e->stream) != hipSuccess) rc = fail(DPGO_HIP_EDEVICE, "sync");
    if (rc != DPGO_HIP_OK) return bail(rc);
  }
  *out = e;
  return DPGO_HIP_OK;
}

int dpgo_rbcd_destroy(dpgo_rbcd e) {
  if (!e) return DPGO_HIP_OK;
  // drain the launch stream (possibly the caller's) and the engine's own; destroy only the own stream
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  hipStream_t own = e->own_stream;
  if (own) (void)hipStreamSynchronize(own);
  delete e;
  if (own) (void)hipStreamDestroy(own);
  return DPGO_HIP_OK;
}

namespace {
void use_stream(dpgo_rbcd e, hipStream_t s) {
  if (e->side) (void)hipStreamSynchronize(e->side);
  e->stream = s;
  for (auto* h : e->prob)
    if (h) h->stream = s;  // verbatim: a NULL stream is the HIP null stream here
}
}  // namespace

int dpgo_rbcd_set_stream(dpgo_rbcd e, void* stream) {
  if (!e) return fail(DPGO_HIP_EINVAL, "null engine");
  // work already queued on the previous stream completes before anything on the new one
  if (e->stream != static_cast<hipStream_t>(stream)) HIP_TRY(hipStreamSynchronize(e->stream));
  use_stream(e, static_cast<hipStream_t>(stream));
  return DPGO_HIP_OK;
}

int dpgo_rbcd_reset_stream(dpgo_rbcd e) {
  if (!e) return fail(DPGO_HIP_EINVAL, "null engine");
  if (e->stream != e->own_stream) HIP_TRY(hipStreamSynchronize(e->stream));
  use_stream(e, e->own_stream);
  return DPGO_HIP_OK;
}

int dpgo_rbcd_info(dpgo_rbcd e, int* num_colors, int* owned_agents, int* owned_poses, int* per_color) {
  if (!e) return fail(DPGO_HIP_EINVAL, "null engine");
  if (num_colors) *num_colors = e->ncolors;
  if (owned_agents) *owned_agents = static_cast<int>(e->owned.size());
  if (owned_poses) *owned_poses = static_cast<int>(e->Nown);
  if (per_color)
    for (int c = 0; c < e->ncolors; ++c) per_color[c] = e->color_off[c + 1] - e->color_off[c];
  return DPGO_HIP_OK;
}

int dpgo_rbcd_color_of_agent(dpgo_rbcd e, int* color) {
  if (!e || !color) return fail(DPGO_HIP_EINVAL, "null argument");
  std::copy(e->color.begin(), e->color.end(), color);
  return DPGO_HIP_OK;
}

int dpgo_rbcd_exchange_counts(dpgo_rbcd e, long long* send_counts, long long* recv_counts) {
  if (!e) return fail(DPGO_HIP_EINVAL, "null engine");
  for (int p = 0; p < e->world; ++p) {
    if (send_counts) send_counts[p] = e->send_counts[p];
    if (recv_counts) recv_counts[p] = e->recv_counts[p];
  }
  return DPGO_HIP_OK;
}

// The selected colour's updateY / XPrev copy / deferred updateV that dpgo_rbcd_pre_exchange queued on the side stream:
// every entry point that reads or writes Y, V or XPrev joins it first (the launch stream waits on its event).
static int join_side(dpgo_rbcd e) {
  if (e->sel_pending) {
    HIP_TRY(hipStreamWaitEvent(e->stream, e->ev_sel, 0));
    e->sel_pending = false;
  }
  return DPGO_HIP_OK;
}

int dpgo_rbcd_set_X(dpgo_rbcd e, const double* Xg) {
  if (!e || !Xg) return fail(DPGO_HIP_EINVAL, "null argument");
  DPGO_TRY(join_side(e));
  const size_t rbs = e->rb();
  std::vector<double> host(std::max<size_t>(static_cast<size_t>(e->Nown) * rbs, 1));
  for (long q = 0; q < e->Nown; ++q)
    std::memcpy(&host[q * rbs], Xg + static_cast<size_t>(e->own_global[q]) * rbs, sizeof(double) * rbs);
  const size_t bytes = sizeof(double) * e->Nown * rbs;
  if (bytes) {
    HIP_TRY(hipMemcpyAsync(e->X.p, host.data(), bytes, hipMemcpyHostToDevice, e->stream));
    // PGOAgent::setX -> initializeAcceleration (:55-68, :1062-1071): XPrev = V = Y = X
    HIP_TRY(hipMemcpyAsync(e->Y.p, e->X.p, bytes, hipMemcpyDeviceToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(e->V.p, e->X.p, bytes, hipMemcpyDeviceToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(e->Xprev.p, e->X.p, bytes, hipMemcpyDeviceToDevice, e->stream));
  }
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->gamma = 0.0;
  e->alpha = 0.0;
  e->iteration = 0;
  e->last_color = -1;
  std::fill(e->v_pending.begin(), e->v_pending.end(), 0);
  return DPGO_HIP_OK;
}

int dpgo_rbcd_get_X(dpgo_rbcd e, double* Xg) {
  if (!e || !Xg) return fail(DPGO_HIP_EINVAL, "null argument");
  DPGO_TRY(join_side(e));
  const size_t rbs = e->rb();
  std::vector<double> host(std::max<size_t>(static_cast<size_t>(e->Nown) * rbs, 1));
  if (e->Nown) {
    HIP_TRY(hipMemcpyAsync(host.data(), e->X.p, sizeof(double) * e->Nown * rbs, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
  }
  for (long q = 0; q < e->Nown; ++q)
    std::memcpy(Xg + static_cast<size_t>(e->own_global[q]) * rbs, &host[q * rbs], sizeof(double) * rbs);
  return DPGO_HIP_OK;
}

static bool restart_now(dpgo_rbcd e) {
  return e->P.acceleration && ((e->iteration + 1) % e->P.restart_interval == 0);  // shouldRestart :1033-1038
}

int dpgo_rbcd_pre_exchange(dpgo_rbcd e, int color) {
  if (!e || color < 0 || color >= e->ncolors) return fail(DPGO_HIP_EINVAL, "bad colour");
  DPGO_TRY(join_side(e));  // a second pre_exchange without an update in between
  // With a robust cost the non-selected agents' reweighting reads their own X and, for shared loop closures, the
  // neighbour poses of their dictionaries (snapshot_neighbors at their last selection): nothing here reads the
  // halo, so every colour order (the cyclic schedule, the example's greedy robot) and every rank count give
  // bitwise the same weights.
  e->last_color = color;
  e->iteration += 1;  // mIterationNumber++ (:643)
  // shouldUpdateLoopClosureWeights (:1174-1179): every agent reweights at the start of its iterate;
  // the non-selected ones here, the selected ones in dpgo_rbcd_update once their neighbours' poses
  // of this iteration have arrived (the order of examples/MultiRobotExample.cpp:181-213)
  e->gnc_due = e->P.robust_cost != DPGO_ROBUST_L2 && (e->iteration + 1) % e->P.robust_opt_inner_iters == 0;
  if (e->gnc_due) {
    for (int c = 0; c < e->ncolors; ++c)
      if (c != color) DPGO_TRY(reweight_color(e, c));
    if (e->P.acceleration) {  // initializeAcceleration (:1062-1071): XPrev = V = Y = X, gamma = alpha = 0
      const long bytes = static_cast<long>(sizeof(double)) * e->Nown * static_cast<long>(e->rb());
      if (bytes) {
        HIP_TRY(hipMemcpyAsync(e->Xprev.p, e->X.p, bytes, hipMemcpyDeviceToDevice, e->stream));
        HIP_TRY(hipMemcpyAsync(e->V.p, e->X.p, bytes, hipMemcpyDeviceToDevice, e->stream));
        HIP_TRY(hipMemcpyAsync(e->Y.p, e->X.p, bytes, hipMemcpyDeviceToDevice, e->stream));
      }
      e->gamma = 0.0;
      e->alpha = 0.0;
      std::fill(e->v_pending.begin(), e->v_pending.end(), 0);  // V = X supersedes a deferred updateV
    }
  }
  const bool restart = restart_now(e);
  // XPrev = X (:673): every agent's on a restart iteration (restartNesterovAcceleration reads it);
  // otherwise only the selected colour's, for its status (fused into its combination pass below;
  // without acceleration the update's own select pass compares against the old X in place)
  if (restart) DPGO_TRY(copy_poses(e, e->Xprev.p, e->X.p, 0, e->Nown));
  if (!e->P.acceleration) return DPGO_HIP_OK;
  const double N = static_cast<double>(e->K);
  e->gamma = (1.0 + std::sqrt(1.0 + 4.0 * N * N * e->gamma * e->gamma)) / (2.0 * N);  // updateGamma
  e->alpha = 1.0 / (e->gamma * N);                                                     // updateAlpha
  // N > 1: the selected colour's updateY (which nothing of the halo reads) goes to the side stream, after
  // everything queued so far; the other colours' combinations (whose X the halo sends) stay in order on the
  // launch stream, so the pack and the exchange can start while the side stream works
  hipStream_t on = nullptr;
  if (e->side && e->prob[color]) {
    HIP_TRY(hipEventRecord(e->ev_start, e->stream));
    HIP_TRY(hipStreamWaitEvent(e->side, e->ev_start, 0));
    on = e->side;
  }
  for (int c = 0; c < e->ncolors; ++c) {
    if (!e->prob[c]) continue;
    double* Xc = color_ptr(e, e->X, c);
    double* Yc = color_ptr(e, e->Y, c);
    if (c == color) {
      // updateY (selected); XPrev = X (:673) for the status, written from the same loads (a restart
      // iteration already copied every X above)
      DPGO_TRY(nesterov_comb(e, c, Yc, e->P.status && !restart ? color_ptr(e, e->Xprev, c) : nullptr, on));
      if (on) {
        HIP_TRY(hipEventRecord(e->ev_sel, e->side));
        e->sel_pending = true;
      }
      continue;
    }
    // non-selected agents, iterate(false): updateY, updateX(false, true): X = Y (one fused pass,
    // written to X only: until this agent's next updateY its Y equals X, so the G assembly and the
    // pack read X, and Y is not stored); updateV: V = project(V + gamma (X - Y)) = project(V)
    // because X == Y exactly, and V already lies on the manifold (a previous project() output), so
    // that pass is skipped.  A deferred updateV of this colour's last update runs in the same pass.
    DPGO_TRY(nesterov_comb(e, c, Xc));
    if (restart) {  // restartNesterovAcceleration(false): X = XPrev, V = Y = X (Y implied, as above)
      DPGO_TRY(copy_poses(e, e->X.p, e->Xprev.p, color_first_pose(e, c), color_num_poses(e, c)));
      DPGO_TRY(copy_poses(e, e->V.p, e->X.p, color_first_pose(e, c), color_num_poses(e, c)));
    }
  }
  return DPGO_HIP_OK;
}

int dpgo_rbcd_pack(dpgo_rbcd e, double* send_dev) {
  if (!e) return fail(DPGO_HIP_EINVAL, "null engine");
  if (e->n_send_items == 0) return DPGO_HIP_OK;
  // the aux poses a receiver uses come from agents outside the selected colour, whose Y equals X
  // after dpgo_rbcd_pre_exchange (the others' entries are not read this iteration)
  HIP_TRY(launch_gather_poses(static_cast<int>(e->n_send_items), static_cast<int>(e->rb()), e->pack_idx.p, e->X.p,
                              e->X.p, send_dev, e->stream));
  e->host_bytes += 2.0 * pose_bytes(e) * static_cast<double>(e->n_send_items);
  return DPGO_HIP_OK;
}

// A per-colour halo refreshes only the RX slots the selected colour reads: every read of the halo is the selected
// colour's (its G, its agents' neighbour-pose snapshot; a reweighting reads the dictionaries, not the halo).

int dpgo_rbcd_pack_color(dpgo_rbcd e, int color, double* send_dev) {
  if (!e || color < 0 || color >= e->ncolors) return fail(DPGO_HIP_EINVAL, "bad colour");
  const auto* H = e->halo[color];
  if (H->n_send == 0) return DPGO_HIP_OK;
  HIP_TRY(launch_gather_poses(static_cast<int>(H->n_send), static_cast<int>(e->rb()), H->pack_idx.p, e->X.p, e->X.p,
                              send_dev, e->stream));
  e->host_bytes += 2.0 * pose_bytes(e) * static_cast<double>(H->n_send);
  return DPGO_HIP_OK;
}

int dpgo_rbcd_exchange_counts_color(dpgo_rbcd e, int color, long long* send_counts, long long* recv_counts) {
  if (!e || color < 0 || color >= e->ncolors) return fail(DPGO_HIP_EINVAL, "bad colour");
  for (int p = 0; p < e->world; ++p) {
    if (send_counts) send_counts[p] = e->halo[color]->send_counts[p];
    if (recv_counts) recv_counts[p] = e->halo[color]->recv_counts[p];
  }
  return DPGO_HIP_OK;
}

static int update_body(dpgo_rbcd e, int color, dpgo_opt_result* results);

int dpgo_rbcd_set_selected(dpgo_rbcd e, const int* agent_mask) {
  if (!e) return fail(DPGO_HIP_EINVAL, "null engine");
  if (!agent_mask) {
    e->sel_mask.clear();
    return DPGO_HIP_OK;
  }
  e->sel_mask.assign(e->owned.size(), 0);
  for (size_t q = 0; q < e->owned.size(); ++q) e->sel_mask[q] = agent_mask[e->owned[q]] != 0 ? 1 : 0;
  // the device copy feeds the next update's neighbour snapshot; earlier launches may still read the old one
  DPGO_TRY(join_side(e));
  HIP_TRY(hipStreamSynchronize(e->stream));
  DPGO_TRY(upload_vec(e->sel_mask_dev, e->sel_mask, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return DPGO_HIP_OK;
}

int dpgo_rbcd_update(dpgo_rbcd e, int color, const double* recv_dev, dpgo_opt_result* results) {
  if (!e || color < 0 || color >= e->ncolors) return fail(DPGO_HIP_EINVAL, "bad colour");
  const int rbs = static_cast<int>(e->rb());
  if (e->n_recv_poses > 0) {
    if (!recv_dev) return fail(DPGO_HIP_EINVAL, "receive buffer required");
    HIP_TRY(launch_gather_poses(static_cast<int>(e->n_recv_poses), rbs, e->unpack_x.p, recv_dev, recv_dev, e->RX.p,
                                e->stream));
    e->host_bytes += 2.0 * pose_bytes(e) * static_cast<double>(e->n_recv_poses);
  }
  return update_body(e, color, results);
}

int dpgo_rbcd_update_color(dpgo_rbcd e, int color, const double* recv_dev, dpgo_opt_result* results) {
  if (!e || color < 0 || color >= e->ncolors) return fail(DPGO_HIP_EINVAL, "bad colour");
  const auto* H = e->halo[color];
  if (H->n_recv > 0) {
    if (!recv_dev) return fail(DPGO_HIP_EINVAL, "receive buffer required");
    HIP_TRY(launch_scatter_poses(static_cast<int>(H->n_recv), static_cast<int>(e->rb()), H->unpack_slot.p, recv_dev,
                                 e->RX.p, e->stream));
    e->host_bytes += 2.0 * pose_bytes(e) * static_cast<double>(H->n_recv);
  }
  return update_body(e, color, results);
}

static int update_body(dpgo_rbcd e, int color, dpgo_opt_result* results) {
  DPGO_TRY(join_side(e));  // the selected colour's updateY from the side stream (dpgo_rbcd_pre_exchange)
  const bool restart = restart_now(e);
  // the selected agents now hold their neighbours' poses of this iteration (the halo has arrived)
  if (e->P.robust_cost != DPGO_ROBUST_L2) DPGO_TRY(snapshot_neighbors(e, color));
  if (e->gnc_due) {
    DPGO_TRY(reweight_color(e, color));
    // RobustCost::update (src/DPGO_robust.cpp:86-103): every agent once per reweighting iteration
    if (e->P.robust_cost == DPGO_ROBUST_GNC_TLS && ++e->gnc_iter <= e->P.gnc_max_iters) e->mu *= e->P.gnc_mu_step;
    e->gnc_due = false;
  }
  if (e->prob[color]) {
    double* Xc = color_ptr(e, e->X, color);
    double* Yc = color_ptr(e, e->Y, color);
    double* Pc = color_ptr(e, e->Xprev, color);
    const bool st = e->P.status != 0;
    if (e->P.acceleration) {
      DPGO_TRY(assemble_G(e, color, e->RX.p));  // constructGMatrix(neighborAuxPoseDict)
      DPGO_TRY(optimize_color(e, color, Yc, Xc, results, st && !restart ? Pc : nullptr));
      if (!restart) {
        // updateV: V = project(V + gamma (X - Y)).  Nothing reads this colour's V before its next
        // combination pass (the next dpgo_rbcd_pre_exchange), so it runs inside that pass
        e->v_pending[color] = 1;
        e->v_gamma[color] = e->gamma;
      } else {  // restartNesterovAcceleration(true) (:1040-1060); its V = X supersedes updateV
        DPGO_TRY(copy_poses(e, e->X.p, e->Xprev.p, color_first_pose(e, color), color_num_poses(e, color)));
        DPGO_TRY(assemble_G(e, color, e->RX.p));  // constructGMatrix(neighborPoseDict): same poses
        DPGO_TRY(optimize_color(e, color, Xc, Xc, results, st ? Pc : nullptr));
        DPGO_TRY(copy_poses(e, e->V.p, e->X.p, color_first_pose(e, color), color_num_poses(e, color)));
        DPGO_TRY(copy_poses(e, e->Y.p, e->X.p, color_first_pose(e, color), color_num_poses(e, color)));
      }
    } else {
      DPGO_TRY(assemble_G(e, color, e->RX.p));  // constructGMatrix(neighborPoseDict)
      // in place: the update's final select compares the result against the old X (= XPrev)
      DPGO_TRY(optimize_color(e, color, Xc, Xc, results, st ? Xc : nullptr));
    }
  }
  if (restart) {
    e->gamma = 0.0;
    e->alpha = 0.0;
  }
  return DPGO_HIP_OK;
}

int dpgo_rbcd_central_eval(dpgo_rbcd e, const double* recv_dev, double* f_out, double* gradnorm_sq) {
  if (e) DPGO_TRY(join_side(e));
  if (!e) return fail(DPGO_HIP_EINVAL, "null engine");
  if (e->n_recv_poses > 0) {
    if (!recv_dev) return fail(DPGO_HIP_EINVAL, "receive buffer required");
    HIP_TRY(launch_gather_poses(static_cast<int>(e->n_recv_poses), static_cast<int>(e->rb()), e->unpack_x.p, recv_dev,
                                recv_dev, e->RXc.p, e->stream));
  }
  // per colour: G from the current neighbour poses, then f / |P_X(XQ + G)|^2 / <G, X> per agent.  The example's
  // central evaluation uses the dataset's Q (QCentral, unit weights): under a robust cost the reweighted colour
  // problems evaluate on their unit-weight copy of Q and G is assembled with unit weights.
  const bool unit = e->P.robust_cost != DPGO_ROBUST_L2;
  for (int c = 0; c < e->ncolors; ++c) {
    if (!e->prob[c]) continue;
    DPGO_TRY(assemble_G(e, c, e->RXc.p, unit));
    if (unit)
      DPGO_TRY(eval_sums_unit_dev(e->prob[c], color_ptr(e, e->X, c)));
    else
      DPGO_TRY(eval_sums_dev(e->prob[c], color_ptr(e, e->X, c)));
  }
  double f = 0.0;
  if (gradnorm_sq)
    for (int a = 0; a < e->K; ++a) gradnorm_sq[a] = 0.0;
  for (int c = 0; c < e->ncolors; ++c) {
    if (!e->prob[c]) continue;
    std::vector<double> sums;
    DPGO_TRY(download_sums_public(e->prob[c], sums));
    for (int q = e->color_off[c]; q < e->color_off[c + 1]; ++q) {
      const int a = q - e->color_off[c];
      // central cost: each shared edge's cross term sits in both endpoint agents' <G, X>
      f += sums[a * 4 + 0] - 0.5 * sums[a * 4 + 2];
      if (gradnorm_sq) gradnorm_sq[e->owned[q]] = sums[a * 4 + 1];
    }
  }
  if (f_out) *f_out = f;
  return DPGO_HIP_OK;
}

int dpgo_rbcd_status(dpgo_rbcd e, double* rel_change, int* ready) {
  if (e) DPGO_TRY(join_side(e));
  if (!e) return fail(DPGO_HIP_EINVAL, "null engine");
  for (int c = 0; c < e->ncolors; ++c) {
    dpgo_hip_problem h = e->prob[c];
    if (!h) continue;
    std::vector<AgentState> st(h->K);
    HIP_TRY(hipMemcpyAsync(st.data(), h->state.p, sizeof(AgentState) * h->K, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    for (int q = e->color_off[c]; q < e->color_off[c + 1]; ++q) {
      const AgentState& s = st[q - e->color_off[c]];
      if (rel_change) rel_change[e->owned[q]] = s.status_rel_change;
      if (ready) ready[e->owned[q]] = s.ready;
    }
  }
  return DPGO_HIP_OK;
}

int dpgo_rbcd_stats(dpgo_rbcd e, int* out) {
  if (!e || !out) return fail(DPGO_HIP_EINVAL, "null argument");
  for (int c = 0; c < e->ncolors; ++c) {
    dpgo_hip_problem h = e->prob[c];
    if (!h) continue;
    std::vector<int> st(static_cast<size_t>(h->K) * kStatsInts);
    DPGO_TRY(dpgo_hip_stats(h, st.data()));
    for (int q = e->color_off[c]; q < e->color_off[c + 1]; ++q)
      std::memcpy(out + static_cast<size_t>(e->owned[q]) * kStatsInts, &st[static_cast<size_t>(q - e->color_off[c]) * kStatsInts],
                  sizeof(int) * kStatsInts);
  }
  return DPGO_HIP_OK;
}

// Algorithmic HBM bytes of everything the engine launched so far: the host-counted per-iteration
// passes plus, per agent, each kernel's bytes times the number of launches that did work for the agent
// (from the exact per-agent solver counters).  SURVEY 8(d)'s accounting: an X.Q pass over an agent
// reads its Q as explicit b x b blocks (n + 2 m_in blocks of b^2 8 + 4 B, (n + 1) 4 B of row pointers)
// and the pose vector once; a half pass (each edge once) reads n + m_in blocks.  P = r b 8 B per pose
// vector, Minv / Q_jj packed (b (b + 1) / 2 doubles), S packed (d (d + 1) / 2 doubles).
int dpgo_rbcd_bytes(dpgo_rbcd e, double* bytes, double* evaltcg_bytes_per_color) {
  if (!e) return fail(DPGO_HIP_EINVAL, "null engine");
  const double P = pose_bytes(e), b = e->b, d = e->d;
  const double blk = b * b * 8.0 + 4.0, DW = 8.0 * b * (b + 1) / 2, SW = 8.0 * d * (d + 1) / 2;
  double total = e->host_bytes;
  // the merged tCG iteration (capi.cpp optimize_dev_status): HESS_M also reads r and Minv; k_tcg_updir
  // replaces the update / direction pair and no z vector is written or read
  for (int c = 0; c < e->ncolors; ++c) {
    dpgo_hip_problem h = e->prob[c];
    if (evaltcg_bytes_per_color) evaltcg_bytes_per_color[c] = 0.0;
    if (!h) continue;
    const bool merged = e->P.precon != DPGO_PRECON_EXACT && h->tuning[TUNE_CLASSIC_TCG] == 0 &&
                        h->tuning[TUNE_FUSE_TCG] <= 0;
    const double mx = merged ? P + DW : 0.0;  // HESS_M's extra operands per pose
    std::vector<int> st(static_cast<size_t>(h->K) * kStatsInts);
    DPGO_TRY(dpgo_hip_stats(h, st.data()));
    double calls_all = 0.0;
    for (int a = 0; a < h->K; ++a) {
      const auto& z = e->asz[c][a];
      const int* k = &st[static_cast<size_t>(a) * kStatsInts];
      const double calls = k[0], runs = k[2], iters = k[3], lcon = k[6] + k[7], maxit = k[8], cg = k[10], impl = k[11],
                   full = k[12];
      const double bnd = k[4] + k[5];
      calls_all = std::max(calls_all, calls);
      const double full_in = (z.n + 2.0 * z.m_in) * blk + (z.n + 1.0) * 4.0 + z.n * P;
      const double half_in = (z.n + z.m_in) * blk + (z.n + 1.0) * 4.0 + z.n * P;
      const double gread = z.gslots * P + z.n * 4.0;
      const double evaltcg = full_in + z.n * (SW + DW + P) + gread;  // + grad(x1) when stored (below)
      if (evaltcg_bytes_per_color) evaltcg_bytes_per_color[c] += evaltcg;
      total += calls * evaltcg;
      // first step test: the each-edge-once pass (QF), or the full pass storing Hess[delta] (HESS_QF,
      // counted as taken by agents that continue with CG steps)
      total += (runs - full) * (half_in + z.n * SW) + full * (full_in + z.n * (P + SW + P + mx));
      total += (iters - runs + std::max(0.0, runs - impl - full)) * (full_in + z.n * (P + SW + P + mx));  // HESS
      if (merged) {
        // k_tcg_updir: every explicit step reads delta, Hdelta, eta and writes eta (the first reads no eta);
        // a CG step that continues also reads r, X, Minv and writes r, delta
        total += (cg + bnd - impl) * z.n * 4.0 * P - runs * z.n * P;
        total += std::max(0.0, cg - lcon - maxit) * z.n * (4.0 * P + DW);
      } else {
        // tCG updates: a CG step reads delta, Hdelta, eta, r, X, Minv and writes eta, r, z; a boundary step
        // reads delta, Hdelta, eta and writes eta (the first step of a tCG reads no eta)
        total += cg * z.n * (8.0 * P + DW) - runs * z.n * P + (bnd - impl) * z.n * 4.0 * P;
        total += std::max(0.0, cg - lcon - maxit) * z.n * 3.0 * P;                 // tCG directions
      }
      total += runs * z.n * 3.0 * P + (runs - impl) * z.n * 1.0 * P;            // retraction (+ g)
      total += runs * (half_in + gread);                                          // f(x2)
      if (e->P.status) total += calls * z.n * 2.0 * P;                            // status |X - XPrev|
    }
    // grad(x1) written by EVAL_TCG when stored (per handle, every agent)
    double nposes = 0.0;
    for (const auto& z : e->asz[c]) nposes += z.n;
    total += static_cast<double>(e->g_store_calls[c]) * nposes * P;
    (void)calls_all;
  }
  if (bytes) *bytes = total;
  return DPGO_HIP_OK;
}

// Algorithmic bytes of ONE X.Q launch per SpMM mode over every agent of a colour (the same per-agent
// terms as dpgo_rbcd_bytes): the per-launch figure the in-step roofline divides by the launch time.
static_assert(kSpmmModes == DPGO_SPMM_MODES, "include/dpgo_rbcd.h DPGO_SPMM_MODES != kSpmmModes");

int dpgo_rbcd_mode_bytes(dpgo_rbcd e, int color, double* out) {
  if (!e || !out || color < 0 || color >= e->ncolors) return fail(DPGO_HIP_EINVAL, "bad colour");
  const double P = pose_bytes(e), b = e->b, d = e->d;
  const double blk = b * b * 8.0 + 4.0, DW = 8.0 * b * (b + 1) / 2, SW = 8.0 * d * (d + 1) / 2;
  for (int m = 0; m < kSpmmModes; ++m) out[m] = 0.0;
  for (const auto& z : e->asz[color]) {
    const double full_in = (z.n + 2.0 * z.m_in) * blk + (z.n + 1.0) * 4.0 + z.n * P;
    const double half_in = (z.n + z.m_in) * blk + (z.n + 1.0) * 4.0 + z.n * P;
    const double gread = z.gslots * P + z.n * 4.0;
    out[MODE_EVAL_TCG] += full_in + z.n * (SW + DW + P) + gread;
    out[MODE_HESS] += full_in + z.n * (P + SW + P);
    out[MODE_HESS_QF] += full_in + z.n * (P + SW + P);
    out[MODE_HESS_M] += full_in + z.n * (P + SW + P + P + DW);  // + r, Minv
    out[MODE_HESS_QF_M] += full_in + z.n * (P + SW + P + P + DW);
    out[MODE_QF] += half_in + z.n * SW;
    out[MODE_F] += half_in + gread;
  }
  return DPGO_HIP_OK;
}

int dpgo_rbcd_set_trace(dpgo_rbcd e, int capacity) {
  if (!e) return fail(DPGO_HIP_EINVAL, "null engine");
  for (auto* h : e->prob)
    if (h) DPGO_TRY(dpgo_hip_set_trace(h, capacity));
  return DPGO_HIP_OK;
}

int dpgo_rbcd_get_trace(dpgo_rbcd e, int agent, double* out, int max_records, int* count) {
  if (!e || agent < 0 || agent >= e->K) return fail(DPGO_HIP_EINVAL, "bad agent");
  for (int c = 0; c < e->ncolors; ++c)
    for (int q = e->color_off[c]; q < e->color_off[c + 1]; ++q)
      if (e->owned[q] == agent) return dpgo_hip_get_trace(e->prob[c], q - e->color_off[c], out, max_records, count);
  return fail(DPGO_HIP_EINVAL, "agent not owned by this rank");
}

int dpgo_rbcd_set_tuning(dpgo_rbcd e, int key, int value) {
  if (!e) return fail(DPGO_HIP_EINVAL, "null engine");
  for (auto* h : e->prob)
    if (h) DPGO_TRY(dpgo_hip_problem_set_tuning(h, key, value));
  return DPGO_HIP_OK;
}

int dpgo_rbcd_set_kernel_timing(dpgo_rbcd e, int on) {
  if (!e) return fail(DPGO_HIP_EINVAL, "null engine");
  for (auto* h : e->prob)
    if (h) {
      h->timing = on < 0 ? 0 : on;
      for (auto& q : h->timing_seq) q = 0;
    }
  return DPGO_HIP_OK;
}

int dpgo_rbcd_kernel_times_ex(dpgo_rbcd e, double* ms_per_mode, long long* launches_per_mode, double* batch_equiv) {
  if (!e) return fail(DPGO_HIP_EINVAL, "null engine");
  double frac[kSpmmModes] = {};
  for (auto* h : e->prob)
    if (h) DPGO_TRY(take_spmm_times(h, e->spmm_ms, e->spmm_launches, frac));
  for (int m = 0; m < kSpmmModes; ++m) {
    if (ms_per_mode) ms_per_mode[m] = e->spmm_ms[m];
    if (launches_per_mode) launches_per_mode[m] = e->spmm_launches[m];
    if (batch_equiv) batch_equiv[m] = frac[m];
    e->spmm_ms[m] = 0.0;
    e->spmm_launches[m] = 0;
  }
  return DPGO_HIP_OK;
}

int dpgo_rbcd_kernel_times(dpgo_rbcd e, double* ms_per_mode, long long* launches_per_mode) {
  return dpgo_rbcd_kernel_times_ex(e, ms_per_mode, launches_per_mode, nullptr);
}

int dpgo_rbcd_bench_spmm(dpgo_rbcd e, int color, int reps, double* bytes, double* ms) {
  if (!e || color < 0 || color >= e->ncolors) return fail(DPGO_HIP_EINVAL, "bad colour");
  dpgo_hip_problem h = e->prob[color];
  if (!h) {
    if (bytes) *bytes = 0.0;
    if (ms) *ms = 0.0;
    return DPGO_HIP_OK;
  }
  if (bytes) *bytes = dpgo_hip_spmm_bytes(h);
  DPGO_TRY(ensure_work_public(h));
  return dpgo_hip_bench_spmm(h, color_ptr(e, e->X, color), h->tA.p, reps, ms);
}

int dpgo_rbcd_spmm_bytes(dpgo_rbcd e, int color, double* bsr_bytes, double* format_bytes) {
  if (!e || color < 0 || color >= e->ncolors) return fail(DPGO_HIP_EINVAL, "bad colour");
  dpgo_hip_problem h = e->prob[color];
  if (bsr_bytes) *bsr_bytes = h ? dpgo_hip_spmm_bytes_bsr(h) : 0.0;
  if (format_bytes) *format_bytes = h ? dpgo_hip_spmm_bytes(h) : 0.0;
  return DPGO_HIP_OK;
}

int dpgo_rbcd_bench_hvp(dpgo_rbcd e, int color, int reps, double* ms) {
  if (!e || color < 0 || color >= e->ncolors) return fail(DPGO_HIP_EINVAL, "bad colour");
  dpgo_hip_problem h = e->prob[color];
  if (!h) {
    if (ms) *ms = 0.0;
    return DPGO_HIP_OK;
  }
  DPGO_TRY(ensure_work_public(h));
  return dpgo_hip_bench_hvp(h, color_ptr(e, e->X, color), h->tA.p, h->tB.p, reps, ms);
}

int dpgo_rbcd_counters(dpgo_rbcd e, long long* agent_updates, long long* iterations) {
  if (!e) return fail(DPGO_HIP_EINVAL, "null engine");
  if (agent_updates) *agent_updates = e->agent_updates;
  if (iterations) *iterations = e->iteration;
  return DPGO_HIP_OK;
}

}  // extern "C"

// ---- native halo exchange over RCCL (examples/MultiRobotExample.cpp:188-213: every agent sends its
// public poses to its neighbours before the selected agents update) ---------------------------------
// RCCL is resolved at run time: the copy already in the process when there is one (the loader matches
// its soname, so a caller that created the communicator and this library use the same instance),
// otherwise the system librccl.  Nothing here links RCCL, so the library loads without it.
static_assert(sizeof(ncclUniqueId) == DPGO_RCCL_ID_BYTES, "DPGO_RCCL_ID_BYTES != sizeof(ncclUniqueId)");

namespace {
struct RcclApi {
  void* lib = nullptr;
  std::string err;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommCount)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*CommUserRank)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

RcclApi& rccl() {
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    api.lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL | RTLD_NOLOAD);
    if (!api.lib) api.lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!api.lib) api.lib = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!api.lib) {
      const char* e = dlerror();
      api.err = e ? e : "librccl.so.1 not found";
      return;
    }
#define DPGO_RCCL_SYM(f) api.f = reinterpret_cast<decltype(api.f)>(dlsym(api.lib, "nccl" #f))
    DPGO_RCCL_SYM(GetUniqueId);
    DPGO_RCCL_SYM(CommInitRank);
    DPGO_RCCL_SYM(CommDestroy);
    DPGO_RCCL_SYM(CommCount);
    DPGO_RCCL_SYM(CommUserRank);
    DPGO_RCCL_SYM(Send);
    DPGO_RCCL_SYM(Recv);
    DPGO_RCCL_SYM(GroupStart);
    DPGO_RCCL_SYM(GroupEnd);
    DPGO_RCCL_SYM(GetErrorString);
#undef DPGO_RCCL_SYM
    if (!api.GetUniqueId || !api.CommInitRank || !api.CommDestroy || !api.CommCount || !api.CommUserRank ||
        !api.Send || !api.Recv || !api.GroupStart || !api.GroupEnd || !api.GetErrorString) {
      api.err = "librccl.so.1 lacks a required entry point";
      api.lib = nullptr;
    }
  });
  return api;
}

int rccl_check(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return DPGO_HIP_OK;
  return fail(DPGO_HIP_EDEVICE, std::string(what) + ": " + rccl().GetErrorString(r));
}

int rccl_ready() {
  if (!rccl().lib) return fail(DPGO_HIP_EDEVICE, "RCCL unavailable: " + rccl().err);
  return DPGO_HIP_OK;
}
}  // namespace

dpgo_rbcd_s::~dpgo_rbcd_s() {
  if (comm && own_comm && rccl().lib) (void)rccl().CommDestroy(comm);
  if (side) {
    (void)hipStreamSynchronize(side);
    (void)hipStreamDestroy(side);
  }
  if (ev_start) (void)hipEventDestroy(ev_start);
  if (ev_sel) (void)hipEventDestroy(ev_sel);
  release();
}

int dpgo_rccl_unique_id(void* id_out) {
  if (!id_out) return fail(DPGO_HIP_EINVAL, "null argument");
  DPGO_TRY(rccl_ready());
  ncclUniqueId id;
  DPGO_TRY(rccl_check(rccl().GetUniqueId(&id), "ncclGetUniqueId"));
  std::memcpy(id_out, &id, sizeof(id));
  return DPGO_HIP_OK;
}

int dpgo_rbcd_comm_init(dpgo_rbcd e, const void* id) {
  if (!e || !id) return fail(DPGO_HIP_EINVAL, "null argument");
  if (e->comm) return fail(DPGO_HIP_ESTATE, "engine already has a communicator");
  DPGO_TRY(rccl_ready());
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  ncclComm_t c = nullptr;
  DPGO_TRY(rccl_check(rccl().CommInitRank(&c, e->world, uid, e->rank), "ncclCommInitRank"));
  e->comm = c;
  e->own_comm = true;
  return DPGO_HIP_OK;
}

int dpgo_rbcd_exact_factor_info(dpgo_rbcd e, int color, long long* nodes, int* levels, int* max_s_tiles,
                                long long* panel_doubles, double* factor_ms, int* factor_count) {
  if (!e || color < 0 || color >= e->ncolors) return fail(DPGO_HIP_EINVAL, "bad colour");
  if (!e->prob[color]) {
    if (nodes) *nodes = 0;
    if (levels) *levels = 0;
    if (max_s_tiles) *max_s_tiles = 0;
    if (panel_doubles) *panel_doubles = 0;
    if (factor_ms) *factor_ms = 0.0;
    if (factor_count) *factor_count = 0;
    return DPGO_HIP_OK;
  }
  return dpgo_hip_exact_factor_info(e->prob[color], nodes, levels, max_s_tiles, panel_doubles, factor_ms, factor_count);
}

int dpgo_rbcd_bench_precond(dpgo_rbcd e, int color, int reps, double* ms_fwd, double* ms_bwd, double* panel_bytes) {
  if (!e || color < 0 || color >= e->ncolors) return fail(DPGO_HIP_EINVAL, "bad colour");
  if (!e->prob[color]) {
    if (ms_fwd) *ms_fwd = 0.0;
    if (ms_bwd) *ms_bwd = 0.0;
    if (panel_bytes) *panel_bytes = 0.0;
    return DPGO_HIP_OK;
  }
  DPGO_TRY(join_side(e));
  return dpgo_hip_bench_precond(e->prob[color], color_ptr(e, e->X, color), reps, ms_fwd, ms_bwd, panel_bytes);
}

int dpgo_rbcd_exact_sweep_bytes(dpgo_rbcd e, int color, double* fwd_bytes, double* bwd_bytes) {
  if (!e || color < 0 || color >= e->ncolors || !fwd_bytes || !bwd_bytes) return fail(DPGO_HIP_EINVAL, "bad argument");
  if (!e->prob[color]) {
    *fwd_bytes = *bwd_bytes = 0.0;
    return DPGO_HIP_OK;
  }
  return dpgo_hip_exact_sweep_bytes(e->prob[color], fwd_bytes, bwd_bytes);
}

int dpgo_rbcd_exact_factor_flops(dpgo_rbcd e, int color, double* cholesky_flops, double* inverse_flops) {
  if (!e || color < 0 || color >= e->ncolors || !cholesky_flops || !inverse_flops) return fail(DPGO_HIP_EINVAL, "bad argument");
  if (!e->prob[color]) {
    *cholesky_flops = *inverse_flops = 0.0;
    return DPGO_HIP_OK;
  }
  return dpgo_hip_exact_factor_flops(e->prob[color], cholesky_flops, inverse_flops);
}

int dpgo_rbcd_comm_info(dpgo_rbcd e, int* count, int* rank) {
  if (!e || !count || !rank) return fail(DPGO_HIP_EINVAL, "null argument");
  *count = -1;
  *rank = -1;
  if (!e->comm) return DPGO_HIP_OK;
  DPGO_TRY(rccl_check(rccl().CommCount(e->comm, count), "ncclCommCount"));
  DPGO_TRY(rccl_check(rccl().CommUserRank(e->comm, rank), "ncclCommUserRank"));
  return DPGO_HIP_OK;
}

int dpgo_rbcd_comm_attach(dpgo_rbcd e, void* comm) {
  if (!e || !comm) return fail(DPGO_HIP_EINVAL, "null argument");
  if (e->comm) return fail(DPGO_HIP_ESTATE, "engine already has a communicator");
  DPGO_TRY(rccl_ready());
  int count = 0, me = -1;
  DPGO_TRY(rccl_check(rccl().CommCount(static_cast<ncclComm_t>(comm), &count), "ncclCommCount"));
  DPGO_TRY(rccl_check(rccl().CommUserRank(static_cast<ncclComm_t>(comm), &me), "ncclCommUserRank"));
  if (count != e->world || me != e->rank) return fail(DPGO_HIP_EINVAL, "communicator does not match the engine's ranks");
  e->comm = static_cast<ncclComm_t>(comm);
  e->own_comm = false;
  return DPGO_HIP_OK;
}

namespace {
// one RCCL group: every peer's send and receive of a plan, on the engine stream (stream order = halo order)
int rccl_halo(dpgo_rbcd e, const std::vector<long long>& sc, const std::vector<long long>& so,
              const std::vector<long long>& rcn, const std::vector<long long>& ro) {
  DPGO_TRY(rccl_check(rccl().GroupStart(), "ncclGroupStart"));
  int rc = DPGO_HIP_OK;
  for (int p = 0; p < e->world && rc == DPGO_HIP_OK; ++p) {
    if (sc[p] > 0)
      rc = rccl_check(rccl().Send(e->xsend.p + so[p], static_cast<size_t>(sc[p]), ncclFloat64, p, e->comm, e->stream),
                      "ncclSend");
    if (rc == DPGO_HIP_OK && rcn[p] > 0)
      rc = rccl_check(rccl().Recv(e->xrecv.p + ro[p], static_cast<size_t>(rcn[p]), ncclFloat64, p, e->comm, e->stream),
                      "ncclRecv");
  }
  const int rc_end = rccl_check(rccl().GroupEnd(), "ncclGroupEnd");
  DPGO_TRY(rc);
  return rc_end;
}
}  // namespace

int dpgo_rbcd_exchange(dpgo_rbcd e, const double** recv_dev) {
  if (!e || !recv_dev) return fail(DPGO_HIP_EINVAL, "null argument");
  if (e->world > 1 && !e->comm) return fail(DPGO_HIP_ESTATE, "no communicator (dpgo_rbcd_comm_init / _attach)");
  HIP_TRY(e->xsend.ensure(std::max<long long>(e->send_off[e->world], 1)));
  HIP_TRY(e->xrecv.ensure(std::max<long long>(e->recv_off[e->world], 1)));
  DPGO_TRY(dpgo_rbcd_pack(e, e->xsend.p));
  if (e->world > 1) DPGO_TRY(rccl_halo(e, e->send_counts, e->send_off, e->recv_counts, e->recv_off));
  *recv_dev = e->xrecv.p;
  return DPGO_HIP_OK;
}

int dpgo_rbcd_exchange_color(dpgo_rbcd e, int color, const double** recv_dev) {
  if (!e || !recv_dev || color < 0 || color >= e->ncolors) return fail(DPGO_HIP_EINVAL, "bad argument");
  if (e->world > 1 && !e->comm) return fail(DPGO_HIP_ESTATE, "no communicator (dpgo_rbcd_comm_init / _attach)");
  const auto* H = e->halo[color];
  HIP_TRY(e->xsend.ensure(std::max<long long>(e->send_off[e->world], 1)));  // the full plan bounds every colour's
  HIP_TRY(e->xrecv.ensure(std::max<long long>(e->recv_off[e->world], 1)));
  DPGO_TRY(dpgo_rbcd_pack_color(e, color, e->xsend.p));
  if (e->world > 1) DPGO_TRY(rccl_halo(e, H->send_counts, H->send_off, H->recv_counts, H->recv_off));
  *recv_dev = e->xrecv.p;
  return DPGO_HIP_OK;
}

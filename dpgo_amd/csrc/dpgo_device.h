// Device-side building blocks shared by the DPGO HIP kernels (gfx950 / CDNA4, fp64).
//
// Lane mapping used by every per-pose kernel ("pose quad"):
//   a 64-lane wavefront handles 16 poses; the 4 lanes of a DPP quad belong to one pose and
//   lane k = lane & 3 owns column k of the r x (d+1) pose block X_j = [Y_j | p_j]
//   (column-major, so column k is r contiguous doubles).  For d = 2 (b = 3) lane 3 of each
//   quad is idle.  A workgroup of 256 threads (4 waves) covers one tile of 64 poses.
// Cross-lane traffic inside a quad uses DPP quad_perm moves (no LDS).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dpgo {

typedef double f64x2 __attribute__((ext_vector_type(2)));

constexpr int kThreads = 256;
constexpr int kPosesPerWave = 16;
constexpr int kTilePoses = 64;

// ---- per-agent scalar state of the on-device RTR / tCG state machine -------------------
struct AgentState {
  double f1, ngf, f2, ngf2;       // cost / Riemannian-gradient norm at x1 and at x2
  double f_init, ngf_init;        // statistics before optimisation
  double Delta, Delta_max;        // trust-region radius
  double e_Pe, e_Pd, d_Pd, z_r;   // tCG recurrences
  double norm_r0, alpha, tau, beta, step;
  double g_eta, eta_Heta, rho, rel_change;  // eta_Heta: carried through tCG as a scalar (OP_TCG_CHECK)
  double d_Hd;                              // <delta, Hdelta> of the last step test
  double r_stop;  // tCG stopping threshold |r_0| min(|r_0|^theta, kappa), set with |r_0|
  int tcg_active;   // tCG still iterating
  int tcg_mode;     // update kernel: 0 CG step (alpha), 1 boundary step (tau) + stop, 2 idle
  int tcg_status;   // 0 NEGCURVTURE 1 EXCREGION 2 LCON 3 SCON 4 MAXITER, -1 none
  int tcg_iters;    // inner iterations of the last tCG
  int run_active;   // participates in the current RTR Run
  int accepted;     // last step accepted (rho > 0.1)
  int runs;         // number of Run() calls (rejection retries)
  int outer_iters;  // accepted + rejected outer iterations
  int gave_up;      // too many rejections -> returns the input
  int copy_pending;  // multi-iteration Run: accepted step still to be copied into x1
  int eta_implicit;  // tCG stopped at its first step on the boundary: eta = step delta is not
                     // materialised (k_retract reads delta; g_eta / eta_Heta set by OP_TCG_STEP)
  int ready;         // PGOAgentStatus::readyToTerminate of the last update (OP_STATUS)
  int r_stop_lcon;   // the threshold's kind: kappa < |r_0|^theta (LCON) or not (SCON)
  int eh_pending;    // merged tCG: a k_tcg_updir left <eta_old, Hdelta> partials (FinalizeArgs::pc) that the
                     // next OP_TCG_STEP_CHECK / OP_RHO folds into eta_Heta with step and d_Hd
  double status_rel_change;  // PGOAgentStatus::relativeChange = |X - XPrev| / sqrt(n) (OP_STATUS)
  // cumulative statistics since the handle was created (never reset; read by dpgo_hip_stats)
  int st_calls;      // optimize calls in which the agent was enabled
  int st_early;      // ... that returned at once (|grad| < tol, src/QuadraticOptimizer.cpp:68-70)
  int st_runs;       // RTR Runs (radius-shrink retries included)
  int st_tcg_iters;  // tCG inner iterations over all Runs
  int st_status[5];  // tCG exits per TcgStatus over all Runs
  int st_gave_up;    // updates that gave up after 12 rejected Runs
  int st_cg_steps;   // tCG step tests that took a CG step (alpha)
  int st_implicit;   // Runs whose tCG ended at its first step on the boundary (eta implicit)
  int st_first_full; // Runs whose first step test was the full pass (MODE_HESS_QF, Hess[delta] stored)
  int trace_n;       // per-iteration trace records written (FinalizeArgs::trace)
};
constexpr int kStatsInts = 13;  // st_calls .. st_first_full, contiguous

// ---- DPP quad helpers -------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long l = __double_as_longlong(v);
  int lo = static_cast<int>(l);
  int hi = static_cast<int>(l >> 32);
  lo = __builtin_amdgcn_mov_dpp(lo, CTRL, 0xF, 0xF, false);
  hi = __builtin_amdgcn_mov_dpp(hi, CTRL, 0xF, 0xF, false);
  return __longlong_as_double((static_cast<long long>(hi) << 32) |
                              static_cast<unsigned int>(lo));
}

// broadcast lane K of the quad to all 4 lanes
template <int K>
__device__ __forceinline__ double qbcast(double v) {
  return dpp_f64<K | (K << 2) | (K << 4) | (K << 6)>(v);
}

// sum over the 4 lanes of the quad; every lane gets the bitwise-identical result
__device__ __forceinline__ double qsum(double v) {
  v += dpp_f64<0xB1>(v);  // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);  // quad_perm [2,3,0,1]
  return v;
}

// deterministic full-wave sum (butterfly); every lane gets the total
// value of lane l + 32 (lanes 0-31; gfx950 v_permlane32_swap on both halves of the double)
__device__ __forceinline__ double lane_plus32(double v) {
  const long long l = __double_as_longlong(v);
  const int lo = static_cast<int>(l), hi = static_cast<int>(l >> 32);
  const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return __longlong_as_double((static_cast<long long>(b[1]) << 32) | static_cast<unsigned int>(a[1]));
}
// value of lane l + 16 (lanes of rows 0 and 2; v_permlane16_swap)
__device__ __forceinline__ double lane_plus16(double v) {
  const long long l = __double_as_longlong(v);
  const int lo = static_cast<int>(l), hi = static_cast<int>(l >> 32);
  const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __longlong_as_double((static_cast<long long>(b[1]) << 32) | static_cast<unsigned int>(a[1]));
}

// Sum over each row of 16 lanes, every lane of the row getting it: __shfl_xor's butterfly (partners l ^ 1, ^ 2, ^ 4,
// ^ 8) bitwise, from DPP moves instead of eight ds_bpermute per double.  After each step both lanes of a pair hold
// the same value, so the row_half_mirror partner (7 - l, the other quad of the 8) and the row_mirror partner (15 - l,
// the other 8 of the row) add the same two numbers as the xor partners (IEEE addition commutes).
__device__ __forceinline__ double row16_sum(double v) {
  v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]: l ^ 1
  v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]: l ^ 2
  v += dpp_f64<0x141>(v);  // row_half_mirror
  v += dpp_f64<0x140>(v);  // row_mirror
  return v;
}
// value of lane l ^ 16 / l ^ 32 (__shfl_xor(v, 16 / 32)) from one v_permlane16_swap / v_permlane32_swap per half
__device__ __forceinline__ double lane_xor16(double v) {
  const long long l = __double_as_longlong(v);
  const int lo = static_cast<int>(l), hi = static_cast<int>(l >> 32);
  const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);  // [0]: rows (0,0,2,2), [1]: rows (1,1,3,3)
  const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const bool odd = (__lane_id() >> 4) & 1;
  const int rl = odd ? a[0] : a[1], rh = odd ? b[0] : b[1];
  return __longlong_as_double((static_cast<long long>(rh) << 32) | static_cast<unsigned int>(rl));
}
__device__ __forceinline__ double lane_xor32(double v) {
  const long long l = __double_as_longlong(v);
  const int lo = static_cast<int>(l), hi = static_cast<int>(l >> 32);
  const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);  // [0]: halves (0,0), [1]: halves (1,1)
  const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  const bool up = __lane_id() >= 32;
  const int rl = up ? a[0] : a[1], rh = up ? b[0] : b[1];
  return __longlong_as_double((static_cast<long long>(rh) << 32) | static_cast<unsigned int>(rl));
}

// Sum over the 64 lanes, valid in LANE 0 ONLY: the halving tree lane 0 sees with __shfl_down or
// __shfl_xor (v_l + v_{l+32}, then + 16, 8, 4, 2, 1) -- the same additions in the same order, so bitwise
// the same -- from two permlane swaps and four DPP row shifts (row_shl:n, lane l reads l + n) instead of
// twelve ds_bpermute round trips.
__device__ __forceinline__ double wave_sum(double v) {
  v += lane_plus32(v);
  v += lane_plus16(v);
  v += dpp_f64<0x108>(v);
  v += dpp_f64<0x104>(v);
  v += dpp_f64<0x102>(v);
  v += dpp_f64<0x101>(v);
  return v;
}


// ---- double-double (hi + lo, |lo| <= ulp(hi) / 2): exact products and compensated sums for the merged
// tCG iteration's one-step polynomials, whose terms cancel by the tCG's residual drop (kernels.hip,
// merged_stop_test).  Error-free transformations: two_sum (Knuth), two_prod (FMA).  Nothing here may be
// reassociated (hipcc does not: no fast-math).  FP contraction is off in these bodies: hipcc contracts a * b + c into an FMA by default, and inside an
// error-free transformation that silently changes what the low part measures (a product contracted into
// two_sum's sum and again into its error term counts the product's rounding error twice).
struct dd {
  double hi, lo;
};
__device__ __forceinline__ dd dd_fast2(double a, double b) {  // |a| >= |b|
#pragma clang fp contract(off)
  const double s = a + b;
  return {s, b - (s - a)};
}
__device__ __forceinline__ dd dd_two_sum(double a, double b) {
#pragma clang fp contract(off)
  const double s = a + b, bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
__device__ __forceinline__ dd dd_add(dd x, dd y) {
#pragma clang fp contract(off)
  const dd s = dd_two_sum(x.hi, y.hi);
  return dd_fast2(s.hi, s.lo + (x.lo + y.lo));
}
// x + a b with the product exact
__device__ __forceinline__ dd dd_fma(dd x, double a, double b) {
#pragma clang fp contract(off)
  const double p = a * b;
  return dd_add(x, {p, __builtin_fma(a, b, -p)});
}
__device__ __forceinline__ dd dd_mul_d(dd x, double a) {
#pragma clang fp contract(off)
  const double p = x.hi * a;
  return dd_fast2(p, __builtin_fma(x.hi, a, -p) + x.lo * a);
}
__device__ __forceinline__ double dd_val(dd x) { return x.hi + x.lo; }

// wave_sum in double-double (same pairs, same order; valid in lane 0 only)
__device__ __forceinline__ dd wave_sum_dd(dd v) {
  v = dd_add(v, {lane_plus32(v.hi), lane_plus32(v.lo)});
  v = dd_add(v, {lane_plus16(v.hi), lane_plus16(v.lo)});
  v = dd_add(v, {dpp_f64<0x108>(v.hi), dpp_f64<0x108>(v.lo)});
  v = dd_add(v, {dpp_f64<0x104>(v.hi), dpp_f64<0x104>(v.lo)});
  v = dd_add(v, {dpp_f64<0x102>(v.hi), dpp_f64<0x102>(v.lo)});
  v = dd_add(v, {dpp_f64<0x101>(v.hi), dpp_f64<0x101>(v.lo)});
  return v;
}

// Reduce-scatter over the quad: lane k ends with col = sum over the 4 lanes of acc[:, k].  Round 1
// (lanes k, k^1) sums the two columns of k's parity, round 2 (lanes k, k^2) column k: the same
// additions in the same order as qsum, so the result equals qsum's bitwise.
template <int R, int B>
__device__ __forceinline__ void quad_reduce_scatter(const double (&acc)[R][B], int k, double (&col)[R]) {
  const bool odd = (k & 1) != 0, hi = (k & 2) != 0;
#pragma unroll
  for (int a = 0; a < R; ++a) {
    const double c0 = acc[a][0], c1 = acc[a][1], c2 = acc[a][2];
    const double c3 = B > 3 ? acc[a][B > 3 ? 3 : 0] : 0.0;
    const double hA = (odd ? c1 : c0) + dpp_f64<0xB1>(odd ? c0 : c1);
    const double hB = (odd ? c3 : c2) + dpp_f64<0xB1>(odd ? c2 : c3);
    col[a] = (hi ? hB : hA) + dpp_f64<0x4E>(hi ? hA : hB);
  }
}

// The same reduce-scatter for an XOR-rotated accumulator (b = 4): lane k keeps column s ^ k of its partial
// sums in slot s, so the partner k ^ x holds column k in slot x and no lane has to select which column
// to send: col = (slot 0 + (k^1)'s slot 1) + (k^2)'s (slot 2 + (k^3)'s slot 3).  Those are qsum's pairs in
// qsum's order, so the result is bitwise quad_reduce_scatter's on the unrotated accumulator.
template <int R>
__device__ __forceinline__ void quad_reduce_scatter_rot(const double (&acc)[R][4], double (&col)[R]) {
#pragma unroll
  for (int a = 0; a < R; ++a) {
    const double lo = acc[a][0] + dpp_f64<0xB1>(acc[a][1]);
    const double hi = acc[a][2] + dpp_f64<0xB1>(acc[a][3]);
    col[a] = lo + dpp_f64<0x4E>(hi);
  }
}

// Y block (first D columns) of a pose on every lane of its quad: full[a][c] = column c of lane c.
template <int R, int D>
__device__ __forceinline__ void quad_gather_y(const double (&col)[R], double (&full)[R][D]) {
#pragma unroll
  for (int a = 0; a < R; ++a) {
    full[a][0] = qbcast<0>(col[a]);
    full[a][1] = qbcast<1>(col[a]);
    if constexpr (D > 2) full[a][D > 2 ? 2 : 0] = qbcast<2>(col[a]);
  }
}

// S = sym(Y^T M_Y) from lane-held columns of M: lane q computes T[:, q] = Y^T M[:, q], the quad
// shares T, and every lane forms S (same FMA chains as sym_ytm).
template <int R, int D>
__device__ __forceinline__ void sym_ytm_cols(const double (&Y)[R][D], const double (&mcol)[R],
                                             double (&S)[D][D]) {
  double Tk[D];
#pragma unroll
  for (int p = 0; p < D; ++p) {
    double s = 0.0;
#pragma unroll
    for (int a = 0; a < R; ++a) s = fma(Y[a][p], mcol[a], s);
    Tk[p] = s;
  }
  double T[D][D];
#pragma unroll
  for (int p = 0; p < D; ++p) {
    T[p][0] = qbcast<0>(Tk[p]);
    T[p][1] = qbcast<1>(Tk[p]);
    if constexpr (D > 2) T[p][D > 2 ? 2 : 0] = qbcast<2>(Tk[p]);
  }
#pragma unroll
  for (int p = 0; p < D; ++p)
#pragma unroll
    for (int q = 0; q < D; ++q) S[p][q] = 0.5 * (T[p][q] + T[q][p]);
}

// Column k of M - [Y S | 0] from lane k's column of M (k = D, the translation column, passes).
template <int R, int D>
__device__ __forceinline__ void sub_y_times_col(const double (&Y)[R][D], const double (&S)[D][D], int k,
                                                const double (&mcol)[R], double (&out)[R]) {
  double Sk[D];
#pragma unroll
  for (int p = 0; p < D; ++p) {
    double v0 = S[p][0], v1 = S[p][1], v2 = D > 2 ? S[p][D > 2 ? 2 : 0] : 0.0, v3 = 0.0;
    if constexpr (D == 2) v2 = 0.0;
    asm("" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));
    Sk[p] = (k & 2) ? ((k & 1) ? v3 : v2) : ((k & 1) ? v1 : v0);
  }
  const bool proj = k < D;
#pragma unroll
  for (int a = 0; a < R; ++a) {
    double s = mcol[a];
#pragma unroll
    for (int p = 0; p < D; ++p) s = fma(-Y[a][p], Sk[p], s);
    out[a] = proj ? s : mcol[a];
  }
}

// Gather a full pose from per-lane columns: full[a][c] = column c held by lane c.
template <int R, int B>
__device__ __forceinline__ void quad_gather(const double (&col)[R], double (&full)[R][B]) {
#pragma unroll
  for (int a = 0; a < R; ++a) {
    full[a][0] = qbcast<0>(col[a]);
    full[a][1] = qbcast<1>(col[a]);
    full[a][2] = qbcast<2>(col[a]);
    if constexpr (B > 3) full[a][3] = qbcast<3>(col[a]);
  }
}

// Load column k (R doubles) of pose j from a column-major r x (b n) array.
template <int R, int B>
__device__ __forceinline__ void load_col(const double* __restrict__ P, long j, int k, bool ok,
                                         double (&col)[R]) {
  if (ok && k < B) {
    const double* p = P + j * (R * B) + k * R;
#pragma unroll
    for (int a = 0; a < R; ++a) col[a] = p[a];
  } else {
#pragma unroll
    for (int a = 0; a < R; ++a) col[a] = 0.0;
  }
}

// Column k of pose j's Y block only (lanes k < b - 1; the translation lane gets zeros): for operands that
// only enter through quad_gather_y (tangent projections, preconditioner projections)
template <int R, int B>
__device__ __forceinline__ void load_col_y(const double* __restrict__ P, long j, int k, bool ok, double (&col)[R]) {
  if (ok && k < B - 1) {
    const double* p = P + j * (R * B) + k * R;
#pragma unroll
    for (int a = 0; a < R; ++a) col[a] = p[a];
  } else {
#pragma unroll
    for (int a = 0; a < R; ++a) col[a] = 0.0;
  }
}

template <int R, int B>
__device__ __forceinline__ void store_col(double* __restrict__ P, long j, int k, bool ok,
                                          const double (&full)[R][B]) {
  if (ok && k < B) {
    double* p = P + j * (R * B) + k * R;
#pragma unroll
    for (int a = 0; a < R; ++a) {
      double v = full[a][0];
      if (k == 1) v = full[a][1];
      if (k == 2) v = full[a][2];
      if constexpr (B > 3) {
        if (k == 3) v = full[a][3];
      }
      p[a] = v;
    }
  }
}

template <int R, int B>
__device__ __forceinline__ double col_dot(const double (&A)[R][B], const double (&C)[R][B], int k) {
  double s = 0.0;
#pragma unroll
  for (int c = 0; c < B; ++c) {
    if (c == k) {
#pragma unroll
      for (int a = 0; a < R; ++a) s = fma(A[a][c], C[a][c], s);
    }
  }
  return s;
}

// S = sym(Y^T M_Y), Y = first D = B-1 columns
template <int R, int B>
__device__ __forceinline__ void sym_ytm(const double (&X)[R][B], const double (&M)[R][B],
                                        double (&S)[B - 1][B - 1]) {
  constexpr int D = B - 1;
  double T[D][D];
#pragma unroll
  for (int p = 0; p < D; ++p)
#pragma unroll
    for (int q = 0; q < D; ++q) {
      double s = 0.0;
#pragma unroll
      for (int a = 0; a < R; ++a) s = fma(X[a][p], M[a][q], s);
      T[p][q] = s;
    }
#pragma unroll
  for (int p = 0; p < D; ++p)
#pragma unroll
    for (int q = 0; q < D; ++q) S[p][q] = 0.5 * (T[p][q] + T[q][p]);
}

// M_Y <- M_Y - Y S   (tangent projection given S = sym(Y^T M_Y), or Hessian correction)
template <int R, int B>
__device__ __forceinline__ void sub_y_times(const double (&X)[R][B], const double (&S)[B - 1][B - 1],
                                            double (&M)[R][B]) {
  constexpr int D = B - 1;
#pragma unroll
  for (int a = 0; a < R; ++a)
#pragma unroll
    for (int q = 0; q < D; ++q) {
      double s = M[a][q];
#pragma unroll
      for (int p = 0; p < D; ++p) s = fma(-X[a][p], S[p][q], s);
      M[a][q] = s;
    }
}

template <int R, int B>
__device__ __forceinline__ void tangent_project_pose(const double (&X)[R][B], double (&V)[R][B]) {
  double S[B - 1][B - 1];
  sym_ytm<R, B>(X, V, S);
  sub_y_times<R, B>(X, S, V);
}

// Q factor (positive diagonal R) of the R x D matrix M (in place), classical Gram-Schmidt
// applied twice ("twice is enough") -- unique Q for full-rank M, matches Householder + sign fix.
template <int R, int D>
__device__ __forceinline__ void qf_inplace(double (&M)[R][D + 1]) {
#pragma unroll
  for (int q = 0; q < D; ++q) {
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int p = 0; p < q; ++p) {
        double s = 0.0;
#pragma unroll
        for (int a = 0; a < R; ++a) s = fma(M[a][p], M[a][q], s);
#pragma unroll
        for (int a = 0; a < R; ++a) M[a][q] = fma(-s, M[a][p], M[a][q]);
      }
    }
    double nn = 0.0;
#pragma unroll
    for (int a = 0; a < R; ++a) nn = fma(M[a][q], M[a][q], nn);
    const double inv = 1.0 / sqrt(nn);
#pragma unroll
    for (int a = 0; a < R; ++a) M[a][q] *= inv;
  }
}

// Polar factor U V^T of the R x D matrix held in the first D columns of M (in place), via
// one-sided Jacobi SVD (columns rotated pairwise until orthogonal; V accumulated).
template <int R, int D>
__device__ __forceinline__ void polar_inplace(double (&M)[R][D + 1]) {
  double V[D][D];
#pragma unroll
  for (int p = 0; p < D; ++p)
#pragma unroll
    for (int q = 0; q < D; ++q) V[p][q] = (p == q) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 30; ++sweep) {
    bool rotated = false;
#pragma unroll
    for (int p = 0; p < D - 1; ++p) {
#pragma unroll
      for (int q = p + 1; q < D; ++q) {
        double alpha = 0.0, beta = 0.0, gamma = 0.0;
#pragma unroll
        for (int a = 0; a < R; ++a) {
          alpha = fma(M[a][p], M[a][p], alpha);
          beta = fma(M[a][q], M[a][q], beta);
          gamma = fma(M[a][p], M[a][q], gamma);
        }
        if (fabs(gamma) > 1e-17 * sqrt(alpha * beta) && gamma != 0.0) {
          rotated = true;
          const double zeta = (beta - alpha) / (2.0 * gamma);
          const double t = copysign(1.0, zeta) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
          const double c = 1.0 / sqrt(1.0 + t * t);
          const double s = c * t;
#pragma unroll
          for (int a = 0; a < R; ++a) {
            const double mp = M[a][p], mq = M[a][q];
            M[a][p] = c * mp - s * mq;
            M[a][q] = s * mp + c * mq;
          }
#pragma unroll
          for (int a = 0; a < D; ++a) {
            const double vp = V[a][p], vq = V[a][q];
            V[a][p] = c * vp - s * vq;
            V[a][q] = s * vp + c * vq;
          }
        }
      }
    }
    if (!rotated) break;
  }
  // U = M diag(1/sigma); polar = U V^T
  double U[R][D];
#pragma unroll
  for (int q = 0; q < D; ++q) {
    double nn = 0.0;
#pragma unroll
    for (int a = 0; a < R; ++a) nn = fma(M[a][q], M[a][q], nn);
    const double inv = nn > 0.0 ? 1.0 / sqrt(nn) : 0.0;
#pragma unroll
    for (int a = 0; a < R; ++a) U[a][q] = M[a][q] * inv;
  }
#pragma unroll
  for (int a = 0; a < R; ++a)
#pragma unroll
    for (int q = 0; q < D; ++q) {
      double s = 0.0;
#pragma unroll
      for (int p = 0; p < D; ++p) s = fma(U[a][p], V[q][p], s);
      M[a][q] = s;
    }
}

// Polar factor via Newton-Schulz  Y <- Y (3 I - Y^T Y) / 2  when ||Y^T Y - I||_F < 0.7 (singular
// values in [0.54, 1.31], inside the iteration's (0, sqrt 3) basin: at most 9 steps), else
// one-sided Jacobi.  Both converge to the same U V^T (the iteration keeps the singular vectors, so
// Jacobi may also finish a Newton-Schulz run); Newton-Schulz needs only FMAs.
template <int R, int D>
__device__ __forceinline__ void polar_fast(double (&M)[R][D + 1]) {
  bool fallback = true;
#pragma unroll 1
  for (int it = 0; it < 12; ++it) {
    double A[D][D];
    double err = 0.0;
#pragma unroll
    for (int p = 0; p < D; ++p)
#pragma unroll
      for (int q = 0; q < D; ++q) {
        double s = 0.0;
#pragma unroll
        for (int a = 0; a < R; ++a) s = fma(M[a][p], M[a][q], s);
        A[p][q] = s;
        const double e = s - (p == q ? 1.0 : 0.0);
        err = fma(e, e, err);
      }
    if (err < 1e-30) {
      fallback = false;
      break;
    }
    if (it == 0 && !(err < 0.5)) break;
    double T[D][D];
#pragma unroll
    for (int p = 0; p < D; ++p)
#pragma unroll
      for (int q = 0; q < D; ++q) T[p][q] = (p == q ? 1.5 : 0.0) - 0.5 * A[p][q];
#pragma unroll
    for (int a = 0; a < R; ++a) {
      double row[D];
#pragma unroll
      for (int q = 0; q < D; ++q) {
        double s = 0.0;
#pragma unroll
        for (int p = 0; p < D; ++p) s = fma(M[a][p], T[p][q], s);
        row[q] = s;
      }
#pragma unroll
      for (int q = 0; q < D; ++q) M[a][q] = row[q];
    }
    // quadratic convergence: from ||Y^T Y - I||_F <= 1e-10 this step reaches the rounding floor,
    // where the 1e-30 test above may never fire (the floor sits near 1e-31)
    if (err < 1e-20) {
      fallback = false;
      break;
    }
  }
  if (fallback) polar_inplace<R, D>(M);
}

}  // namespace dpgo

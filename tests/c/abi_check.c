/* A plain C caller of libdpgo_hip.so that sizes every array from the include/ headers (what a reference-side
 * binding would do).  Compiled by tests/test_host_native.py (consts mode, no GPU) and
 * tests/test_gpu_abi.py (gpu mode).
 *   abi_check consts : prints the header constants the caller sizes its arrays with
 *   abi_check gpu    : runs two RBCD iterations on a small grid with kernel timing on, then calls every
 *                      per-mode / per-agent array entry point with header-sized arrays followed by canary
 *                      words, and checks that no canary was overwritten. */
#include <stdio.h>
#include <string.h>

#include "dpgo_rbcd.h"

#define CANARY_D (-12345.678)
#define CANARY_LL (0x5A5A5A5A5A5A5A5ALL)
#define CANARY_I (0x5A5A5A5A)
#define NCAN 4

static int fail_rc(const char* what, int rc) {
  fprintf(stderr, "%s failed: %d %s\n", what, rc, dpgo_hip_last_error());
  return 1;
}

int main(int argc, char** argv) {
  if (argc > 1 && strcmp(argv[1], "consts") == 0) {
    printf("DPGO_SPMM_MODES %d\nDPGO_STATS_INTS %d\nDPGO_RCCL_ID_BYTES %d\n", DPGO_SPMM_MODES, DPGO_STATS_INTS,
           DPGO_RCCL_ID_BYTES);
    return 0;
  }
  enum { K = 6, A = 2, NA = A * A * A, R = 5, D = 3 };
  dpgo_graph g = NULL;
  int rc = dpgo_graph_grid3d(K, 0ULL, 0.2, 0.1, &g);
  if (rc) return fail_rc("dpgo_graph_grid3d", rc);
  int aop[K * K * K], ranks[NA];
  rc = dpgo_graph_grid_partition(g, A, aop);
  if (rc) return fail_rc("dpgo_graph_grid_partition", rc);
  memset(ranks, 0, sizeof(ranks));
  dpgo_rbcd_params p;
  dpgo_rbcd_default_params(&p);
  p.r = R;
  dpgo_rbcd e = NULL;
  rc = dpgo_rbcd_create(g, NA, aop, ranks, 0, 1, &p, &e);
  if (rc) return fail_rc("dpgo_rbcd_create", rc);
  static double X[R * (D + 1) * K * K * K];
  double ylift[R * D];
  memset(ylift, 0, sizeof(ylift));
  for (int i = 0; i < D; ++i) ylift[i * R + i] = 1.0; /* r x d column-major, orthonormal columns */
  rc = dpgo_graph_chain_init(g, R, ylift, X);
  if (rc) return fail_rc("dpgo_graph_chain_init", rc);
  rc = dpgo_rbcd_set_X(e, X);
  if (rc) return fail_rc("dpgo_rbcd_set_X", rc);
  rc = dpgo_rbcd_set_kernel_timing(e, 1);
  if (rc) return fail_rc("dpgo_rbcd_set_kernel_timing", rc);
  for (int it = 0; it < 2; ++it) {
    rc = dpgo_rbcd_pre_exchange(e, it % 2);
    if (rc) return fail_rc("dpgo_rbcd_pre_exchange", rc);
    rc = dpgo_rbcd_update(e, it % 2, NULL, NULL);
    if (rc) return fail_rc("dpgo_rbcd_update", rc);
  }
  double ms[DPGO_SPMM_MODES + NCAN], bytes[DPGO_SPMM_MODES + NCAN];
  long long launches[DPGO_SPMM_MODES + NCAN];
  int stats[NA * DPGO_STATS_INTS + NCAN];
  for (int i = 0; i < DPGO_SPMM_MODES + NCAN; ++i) {
    ms[i] = bytes[i] = CANARY_D;
    launches[i] = CANARY_LL;
  }
  for (int i = 0; i < NA * DPGO_STATS_INTS + NCAN; ++i) stats[i] = CANARY_I;
  rc = dpgo_rbcd_kernel_times(e, ms, launches);
  if (rc) return fail_rc("dpgo_rbcd_kernel_times", rc);
  rc = dpgo_rbcd_mode_bytes(e, 0, bytes);
  if (rc) return fail_rc("dpgo_rbcd_mode_bytes", rc);
  rc = dpgo_rbcd_stats(e, stats);
  if (rc) return fail_rc("dpgo_rbcd_stats", rc);
  int bad = 0;
  for (int i = DPGO_SPMM_MODES; i < DPGO_SPMM_MODES + NCAN; ++i)
    bad += (ms[i] != CANARY_D) + (bytes[i] != CANARY_D) + (launches[i] != CANARY_LL);
  for (int i = NA * DPGO_STATS_INTS; i < NA * DPGO_STATS_INTS + NCAN; ++i) bad += stats[i] != CANARY_I;
  long long total = 0;
  for (int i = 0; i < DPGO_SPMM_MODES; ++i) total += launches[i];
  dpgo_rbcd_destroy(e);
  dpgo_graph_destroy(g);
  printf("timed launches %lld, overwritten canaries %d\n", total, bad);
  if (bad) return 2;
  if (total <= 0) return 3;
  printf("canaries ok\n");
  return 0;
}

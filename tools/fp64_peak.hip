// fp64 compute ceilings of this MI355X, for the exact preconditioner's numeric factorisation roofline:
// v_mfma_f64_16x16x4_f64 issued back to back (8 independent accumulators per wave, every SIMD of every CU busy) and
// the VALU's v_fma_f64 (8 independent chains per lane).  Measurement tool only; prints one JSON line.
//   hipcc --offload-arch=gfx950 -O3 -o tools/fp64_peak tools/fp64_peak.hip && ./tools/fp64_peak
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_mfma(int iters, double seed, double* out) {
  const int lane = threadIdx.x & 63;
  const double a = seed + lane * 1e-3, b = seed - lane * 1e-3;
  f64x4 acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = f64x4{0.0, 0.0, 0.0, 0.0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[q], 0, 0, 0);
  }
  double s = 0.0;
#pragma unroll
  for (int q = 0; q < 8; ++q) s += acc[q].x + acc[q].y + acc[q].z + acc[q].w;
  if (s == 12345.678) out[blockIdx.x] = s;  // keeps the loop alive; never true for these operands
}

__global__ __launch_bounds__(256) void k_valu(int iters, double seed, double* out) {
  double x[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) x[q] = seed + q * 1e-7 + threadIdx.x * 1e-9;
  const double m = 0.999999999, c = 1e-12;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = fma(x[q], m, c);
  }
  double s = 0.0;
#pragma unroll
  for (int q = 0; q < 8; ++q) s += x[q];
  if (s == 12345.678) out[blockIdx.x] = s;
}

int main() {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  double* out = nullptr;
  const int blocks = cus * 8;  // 8 workgroups of 4 waves per CU: every SIMD holds 8 waves
  hipMalloc(&out, sizeof(double) * blocks);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4000;
  double tf[2] = {0, 0};
  for (int kind = 0; kind < 2; ++kind) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(e0);
      if (kind == 0)
        k_mfma<<<blocks, 256>>>(iters, 1.0, out);
      else
        k_valu<<<blocks, 256>>>(iters, 1.0, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep > 0 && ms < best) best = ms;
    }
    const double waves = static_cast<double>(blocks) * 4.0;
    // MFMA f64 16x16x4: 16 * 16 * 4 multiply-adds = 2048 flop per wave-instruction; VALU fma: 2 flop per lane
    const double flop = kind == 0 ? waves * iters * 8.0 * 2048.0 : waves * 64.0 * iters * 8.0 * 2.0;
    tf[kind] = flop / (best * 1e-3) / 1e12;
  }
  printf("{\"cus\": %d, \"mfma_f64_16x16x4_tflops\": %.2f, \"valu_fma_f64_tflops\": %.2f}\n", cus, tf[0], tf[1]);
  hipFree(out);
  return 0;
}

// fp64 compute ceilings of this MI355X, for the exact preconditioner's numeric factorisation roofline:
// v_mfma_f64_16x16x4_f64 issued back to back (8 independent accumulators per wave, every SIMD of every CU busy) and
// the VALU's v_fma_f64 (8 independent chains per lane).  Each kernel also reads the shader clock counter (clock64,
// s_memtime) and the constant-rate wall clock (wall_clock64, s_memrealtime) around its loop in wave 0 of block 0, so
// the run reports the clock the chip held under each load and the SIMD cycles per instruction -- which tells an
// under-issued MFMA stream (cycles per MFMA above its issue rate) from a lower clock under MFMA load (same cycles per
// instruction, fewer cycles per second).  Measurement tool only; prints one JSON line.
// Build with the MFMA accumulators in VGPRs (-amdgpu-mfma-vgpr-form): by default the compiler keeps the loop-carried
// accumulators in VGPRs and copies all of them through AGPRs around every iteration's MFMAs (128 v_accvgpr moves per
// 8 MFMAs), which is what round 5's 49 TFLOP/s "ceiling" measured.
//   hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form=1 -o tools/fp64_peak tools/fp64_peak.hip
//   ./tools/fp64_peak
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void k_mfma(int iters, double seed, double* out, long long* clk) {
  const int lane = threadIdx.x & 63;
  const double a = seed + lane * 1e-3, b = seed - lane * 1e-3;
  f64x4 acc[NACC];
#pragma unroll
  for (int q = 0; q < NACC; ++q) acc[q] = f64x4{0.0, 0.0, 0.0, 0.0};
  const long long c0 = clock64(), w0 = wall_clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < NACC; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[q], 0, 0, 0);
  }
  double s = 0.0;
#pragma unroll
  for (int q = 0; q < NACC; ++q) s += acc[q].x + acc[q].y + acc[q].z + acc[q].w;
  const long long c1 = clock64(), w1 = wall_clock64();
  if (s == 12345.678) out[blockIdx.x] = s;  // keeps the loop alive; never true for these operands
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[0] = c1 - c0;
    clk[1] = w1 - w0;
  }
}

__global__ __launch_bounds__(256) void k_valu(int iters, double seed, double* out, long long* clk) {
  double x[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) x[q] = seed + q * 1e-7 + threadIdx.x * 1e-9;
  const double m = 0.999999999, c = 1e-12;
  const long long c0 = clock64(), w0 = wall_clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = fma(x[q], m, c);
  }
  double s = 0.0;
#pragma unroll
  for (int q = 0; q < 8; ++q) s += x[q];
  const long long c1 = clock64(), w1 = wall_clock64();
  if (s == 12345.678) out[blockIdx.x] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[0] = c1 - c0;
    clk[1] = w1 - w0;
  }
}

int main() {
  int dev = 0, cus = 0, wall_khz = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, dev);
  double* out = nullptr;
  long long* clk = nullptr;
  const int wg_per_cu[3] = {8, 8, 2};  // MFMA 8 waves / SIMD; VALU 8; MFMA with 1 wave per SIMD (issue alone)
  hipMalloc(&out, sizeof(double) * cus * 8);
  hipMalloc(&clk, sizeof(long long) * 2);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4000;
  const char* names[4] = {"mfma_f64_16x16x4_8acc_8waves", "valu_fma_f64_8chains_8waves", "mfma_f64_16x16x4_8acc_2waves",
                          "mfma_f64_16x16x4_16acc_8waves"};
  double tf[4] = {0, 0, 0, 0}, ghz[4] = {0, 0, 0, 0}, cpi[4] = {0, 0, 0, 0};
  for (int kind = 0; kind < 4; ++kind) {
    const int blocks = cus * (kind == 2 ? 1 : 8);
    const int nacc = kind == 3 ? 16 : 8;
    float best = 1e30f;
    long long hc[2] = {0, 0};
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(e0);
      if (kind == 1)
        k_valu<<<blocks, 256>>>(iters, 1.0, out, clk);
      else if (kind == 3)
        k_mfma<16><<<blocks, 256>>>(iters, 1.0, out, clk);
      else
        k_mfma<8><<<blocks, 256>>>(iters, 1.0, out, clk);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep > 0 && ms < best) {
        best = ms;
        hipMemcpy(hc, clk, sizeof(hc), hipMemcpyDeviceToHost);
      }
    }
    const double waves = static_cast<double>(blocks) * 4.0;
    // MFMA f64 16x16x4: 16 * 16 * 4 multiply-adds = 2048 flop per wave-instruction; VALU fma: 2 flop per lane
    const double per_wave_instr = static_cast<double>(iters) * (kind == 1 ? 8 : nacc);
    const double flop = kind == 1 ? waves * 64.0 * per_wave_instr * 2.0 : waves * per_wave_instr * 2048.0;
    tf[kind] = flop / (best * 1e-3) / 1e12;
    const double wall_s = static_cast<double>(hc[1]) / (wall_khz * 1e3);
    ghz[kind] = wall_s > 0 ? static_cast<double>(hc[0]) / wall_s / 1e9 : 0.0;
    // SIMD cycles per instruction: the waves sharing a SIMD (blocks * 4 waves / (4 SIMDs * cus)) issue in turn
    const double waves_per_simd = waves / (4.0 * cus);
    cpi[kind] = static_cast<double>(hc[0]) / (per_wave_instr * waves_per_simd);
  }
  printf("{\"cus\": %d, \"wall_clock_khz\": %d, \"mfma_f64_16x16x4_tflops\": %.2f, \"valu_fma_f64_tflops\": %.2f",
         cus, wall_khz, tf[0], tf[1]);
  for (int k = 0; k < 4; ++k)
    printf(", \"%s\": {\"tflops\": %.2f, \"clock_ghz\": %.3f, \"simd_cycles_per_instr\": %.2f}", names[k], tf[k], ghz[k],
           cpi[k]);
  printf("}\n");
  hipFree(out);
  hipFree(clk);
  return 0;
}

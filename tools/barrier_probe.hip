// What a dependency between workgroups costs on this MI355X, for the persistent per-colour tCG kernel:
//   launch : a chain of dependent launches of a small kernel (G workgroups, each reads and writes one double per lane
//            of another workgroup's slot) -- the cost the merged tCG pays per kernel boundary today;
//   grid   : one cooperative launch of G workgroups that run the same phases separated by a spin barrier over all
//            of them (release fence, a device-scope counter, bounded spin, acquire fence);
//   group  : the same with the barrier over groups of G / NG workgroups (agent-level barriers, each group exchanging
//            only inside itself);
//   flags  : no read-modify-write at all: every workgroup stores its phase number into its own slot, workgroup 0
//            polls all the slots (one load per lane) and then stores the phase into a release word every
//            workgroup polls -- three memory round trips instead of G serialised device-scope atomics;
//   cg     : the HIP runtime's own grid barrier, cooperative_groups::this_grid().sync();
//   flags_nofence : the flag barrier without the release / acquire fences (each an L2 write-back / invalidate of
//            the workgroup's XCD): what the synchronisation alone costs -- not a valid barrier for data exchange.
// Every spin is bounded (an abort flag ends every wave), and the grid is sized by the occupancy API and launched
// cooperatively (the runtime refuses a grid that cannot be co-resident).  Measurement tool only; prints one JSON line.
//   hipcc --offload-arch=gfx950 -O3 -o tools/barrier_probe tools/barrier_probe.hip && ./tools/barrier_probe
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::printf("{\"error\": \"%s at line %d\"}\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

constexpr int kThreads = 256;
constexpr unsigned kSpinLimit = 1u << 22;  // ~ seconds of s_sleep: a barrier that never completes aborts instead

__global__ __launch_bounds__(kThreads) void k_touch(int G, int phase, double* buf) {
  const int src = (blockIdx.x + 1 + phase) % G;
  const double v = buf[src * kThreads + threadIdx.x];
  __syncthreads();
  buf[blockIdx.x * kThreads + threadIdx.x] = v + 1.0;
}

__device__ __forceinline__ bool bar_wait(unsigned* count, unsigned target, unsigned* abort_flag) {
  __shared__ int s_abort;
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    int ab = 0;
    while (__hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > kSpinLimit) {
        __hip_atomic_store(abort_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ab = 1;
        break;
      }
      if ((spins & 255) == 0 && __hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        ab = 1;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    s_abort = ab;
  }
  __syncthreads();
  return s_abort != 0;
}

// NG groups of G / NG consecutive workgroups; each phase reads a slot of the next workgroup of the same group
__global__ __launch_bounds__(kThreads) void k_phases(int G, int NG, int phases, double* buf, unsigned* counters,
                                                     unsigned* abort_flag) {
  const int per = G / NG, grp = blockIdx.x / per, g0 = grp * per, me = blockIdx.x - g0;
  if (grp >= NG) return;  // (G a multiple of NG: never)
  for (int ph = 0; ph < phases; ++ph) {
    const int src = g0 + (me + 1 + ph) % per;
    const double v = buf[src * kThreads + threadIdx.x];
    __syncthreads();
    buf[blockIdx.x * kThreads + threadIdx.x] = v + 1.0;
    if (bar_wait(&counters[grp * 32], static_cast<unsigned>(per) * (ph + 1), abort_flag)) return;
  }
}

template <bool FENCE>
__device__ __forceinline__ bool flag_wait(unsigned* slots, unsigned* release, int G, unsigned ph,
                                          unsigned* abort_flag) {
  __shared__ int s_abort;
  __syncthreads();
  if (threadIdx.x == 0) {
    if (FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_store(&slots[blockIdx.x * 16], ph, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  int ab = 0;
  if (blockIdx.x == 0) {  // gather: every lane polls its share of the slots
    for (int x = threadIdx.x; x < G && !ab; x += kThreads) {
      unsigned spins = 0;
      while (__hip_atomic_load(&slots[x * 16], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < ph) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > kSpinLimit) {
          __hip_atomic_store(abort_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ab = 1;
          break;
        }
      }
    }
    if (ab) s_abort = 1;
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(release, ph, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x == 0) {
    unsigned spins = 0;
    ab = 0;
    while (__hip_atomic_load(release, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < ph) {
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 255) == 0 && __hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        ab = 1;
        break;
      }
      if (spins > kSpinLimit) {
        ab = 1;
        break;
      }
    }
    if (FENCE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    s_abort = ab;
  }
  __syncthreads();
  return s_abort != 0;
}

template <bool FENCE>
__global__ __launch_bounds__(kThreads) void k_phases_flags(int G, int phases, double* buf, unsigned* slots,
                                                           unsigned* release, unsigned* abort_flag) {
  for (int ph = 0; ph < phases; ++ph) {
    const int src = (blockIdx.x + 1 + ph) % G;
    const double v = buf[src * kThreads + threadIdx.x];
    __syncthreads();
    buf[blockIdx.x * kThreads + threadIdx.x] = v + 1.0;
    if (flag_wait<FENCE>(slots, release, G, static_cast<unsigned>(ph + 1), abort_flag)) return;
  }
}

__global__ __launch_bounds__(kThreads) void k_phases_cg(int G, int phases, double* buf) {
  auto grid = cooperative_groups::this_grid();
  for (int ph = 0; ph < phases; ++ph) {
    const int src = (blockIdx.x + 1 + ph) % G;
    const double v = buf[src * kThreads + threadIdx.x];
    __syncthreads();
    buf[blockIdx.x * kThreads + threadIdx.x] = v + 1.0;
    grid.sync();
  }
}

int main() {
  int dev = 0, cus = 0, occ = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_phases, kThreads, 0));
  const int maxG = occ * cus;
  double* buf = nullptr;
  unsigned *counters = nullptr, *abort_flag = nullptr;
  CK(hipMalloc(&buf, sizeof(double) * kThreads * maxG));
  CK(hipMalloc(&counters, sizeof(unsigned) * 32 * 16));
  CK(hipMalloc(&abort_flag, sizeof(unsigned)));
  unsigned *slots = nullptr, *release = nullptr;
  CK(hipMalloc(&slots, sizeof(unsigned) * 16 * maxG));
  CK(hipMalloc(&release, sizeof(unsigned) * 16));
  CK(hipMemset(buf, 0, sizeof(double) * kThreads * maxG));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::printf("{\"cus\": %d, \"occupancy_blocks_per_cu\": %d, \"results\": [", cus, occ);
  bool firstrow = true;
  const int Gs[] = {256, 512, 980, 1024};
  for (int G : Gs) {
    if (G > maxG) continue;
    // dependent launch chain
    const int L = 2000;
    for (int w = 0; w < 50; ++w) k_touch<<<G, kThreads, 0, s>>>(G, w, buf);
    CK(hipEventRecord(e0, s));
    for (int w = 0; w < L; ++w) k_touch<<<G, kThreads, 0, s>>>(G, w, buf);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("%s{\"G\": %d, \"kind\": \"launch\", \"us_per_phase\": %.3f}", firstrow ? "" : ", ", G, 1e3 * ms / L);
    firstrow = false;
    for (int NG : {1, 4}) {
      if (G % NG) continue;
      const int P = 2000;
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipMemsetAsync(counters, 0, sizeof(unsigned) * 32 * 16, s));
        CK(hipMemsetAsync(abort_flag, 0, sizeof(unsigned), s));
        int g = G, ng = NG, ph = P;
        void* args[] = {&g, &ng, &ph, &buf, &counters, &abort_flag};
        CK(hipEventRecord(e0, s));
        CK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k_phases), dim3(G), dim3(kThreads), args, 0, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        unsigned ab = 0;
        CK(hipMemcpy(&ab, abort_flag, sizeof(unsigned), hipMemcpyDeviceToHost));
        if (rep == 1)
          std::printf(", {\"G\": %d, \"kind\": \"%s\", \"groups\": %d, \"us_per_phase\": %.3f, \"aborted\": %u}", G,
                      NG == 1 ? "grid" : "group", NG, 1e3 * ms / P, ab);
        if (ab) break;
      }
    }
    {  // the runtime's grid barrier
      const int P = 2000;
      for (int rep = 0; rep < 2; ++rep) {
        int g = G, ph = P;
        void* args[] = {&g, &ph, &buf};
        CK(hipEventRecord(e0, s));
        CK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k_phases_cg), dim3(G), dim3(kThreads), args, 0, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep == 1) std::printf(", {\"G\": %d, \"kind\": \"cg\", \"us_per_phase\": %.3f}", G, 1e3 * ms / P);
      }
    }
    for (int fence = 1; fence >= 0; --fence) {  // flag-array barrier over the whole grid
      const int P = 2000;
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipMemsetAsync(slots, 0, sizeof(unsigned) * 16 * maxG, s));
        CK(hipMemsetAsync(release, 0, sizeof(unsigned) * 16, s));
        CK(hipMemsetAsync(abort_flag, 0, sizeof(unsigned), s));
        int g = G, ph = P;
        void* args[] = {&g, &ph, &buf, &slots, &release, &abort_flag};
        CK(hipEventRecord(e0, s));
        CK(hipLaunchCooperativeKernel(fence ? reinterpret_cast<const void*>(k_phases_flags<true>) : reinterpret_cast<const void*>(k_phases_flags<false>), dim3(G), dim3(kThreads), args, 0,
                                      s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        unsigned ab = 0;
        CK(hipMemcpy(&ab, abort_flag, sizeof(unsigned), hipMemcpyDeviceToHost));
        if (rep == 1)
          std::printf(", {\"G\": %d, \"kind\": \"%s\", \"us_per_phase\": %.3f, \"aborted\": %u}", G, fence ? "flags" : "flags_nofence", 1e3 * ms / P, ab);
        if (ab) break;
      }
    }
  }
  std::printf("]}\n");
  CK(hipFree(buf));
  CK(hipFree(counters));
  CK(hipFree(abort_flag));
  return 0;
}

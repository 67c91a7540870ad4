// Returning-atomic throughput/latency probe for work-queue designs (GPU, diagnostic).
//   hipcc --offload-arch=gfx950 -O3 -o atomic_rate atomic_rate.hip && ./atomic_rate
// 768 workgroups x 8 waves; each wave (lane 0) does K dependent fetch_adds on
//   mode 0: one counter per workgroup, mode 1: one counter per 32 workgroups,
//   mode 2: 8 counters (blockIdx % 8), mode 3: one global counter.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(512) probe(unsigned *ctr, int mode, int k, unsigned *sink) {
  const unsigned lane = threadIdx.x & 63u;
  unsigned idx = mode == 0 ? blockIdx.x : mode == 1 ? blockIdx.x / 32 : mode == 2 ? blockIdx.x % 8 : 0;
  unsigned acc = 0;
  for (int i = 0; i < k; ++i) {
    unsigned r = 0;
    if (lane == 0) r = __hip_atomic_fetch_add(ctr + idx * 64, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    acc += __builtin_amdgcn_readfirstlane(r);
  }
  if (acc == 0xFFFFFFFFu) sink[0] = acc;
}

int main() {
  unsigned *ctr, *sink;
  hipMalloc(&ctr, 1024 * 64 * 4);
  hipMalloc(&sink, 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char *names[] = {"per-WG", "per-32-WG", "8 queues", "1 global"};
  for (int mode = 0; mode < 4; ++mode)
    for (int k : {1, 8, 32}) {
      hipMemset(ctr, 0, 1024 * 64 * 4);
      hipLaunchKernelGGL(probe, dim3(768), dim3(512), 0, 0, ctr, mode, k, sink);
      hipDeviceSynchronize();
      float best = 1e9f;
      for (int rep = 0; rep < 5; ++rep) {
        hipEventRecord(a);
        hipLaunchKernelGGL(probe, dim3(768), dim3(512), 0, 0, ctr, mode, k, sink);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      const double n = 768.0 * 8 * k;
      printf("%-10s k=%2d  %8.2f us  %7.1f M atomics/s  %6.2f ns/atomic/wave-chain\n", names[mode], k,
             best * 1e3, n / (best * 1e-3) / 1e6, best * 1e6 / k);
    }
  return 0;
}

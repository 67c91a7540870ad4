// Does hipExtAnyOrderLaunch let kernels of one stream overlap on gfx950?
// K launches of a one-wave kernel that spins ~5 us (s_memrealtime, 100 MHz), issued
// back to back on one stream with and without the flag (and, for scale, a 1024-
// workgroup version). Overlapping launches finish in ~one kernel time; serialised
// ones in K kernel times.
//   hipcc --offload-arch=gfx950 -O3 any_order_probe.hip -o any_order_probe && ./any_order_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>

__global__ void spin_kernel(unsigned ticks, unsigned *sink) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t0;
  while (t - t0 < ticks) t = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && (unsigned)t == 0xFFFFFFFFu) sink[blockIdx.x] = 1;  // keeps the loop
}

#define CHECK(x)                                                        \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));         \
      return 1;                                                         \
    }                                                                   \
  } while (0)

int main() {
  unsigned *sink;
  CHECK(hipMalloc(&sink, 4096 * sizeof(unsigned)));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const int K = 64;
  const unsigned ticks = 500;  // 5 us
  for (int grid : {1, 1024}) {
    for (int rep = 0; rep < 3; ++rep) {
      for (unsigned flags : {0u, (unsigned)hipExtAnyOrderLaunch}) {
        CHECK(hipEventRecord(a, s));
        for (int k = 0; k < K; ++k)
          hipExtLaunchKernelGGL(spin_kernel, dim3(grid), dim3(64), 0, s, nullptr, nullptr, k ? flags : 0u,
                                ticks, sink);
        CHECK(hipEventRecord(b, s));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        std::printf("grid %4d flags %u: %d launches of a 5 us kernel in %8.1f us (%.2f us each)\n", grid, flags, K,
                    ms * 1e3, ms * 1e3 / K);
      }
    }
  }
  CHECK(hipFree(sink));
  return 0;
}

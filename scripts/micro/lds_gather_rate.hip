// lds_gather_rate.hip -- LDS cost of the decoder's table gathers (measurement
// infrastructure): a 16 KB u16 table of random values in LDS; each lane runs 4
// independent pointer-chasing chains (index = previous value + lane salt), so the
// only per-step VALU is an add and an and. Modes: random ds_read_u16 (the 13-bit
// first-level lookup), the same with ~18 % of lanes active, lane-linear
// (conflict-free), one address per wave (broadcast), ds_bpermute_b32 (random lane),
// random ds_read_b32. Waves per CU 8 / 16 / 24. Prints LDS cycles per
// wave-instruction per CU at the measured rate (2.1 GHz assumed).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kIters = 2048;
constexpr int kChains = 4;

template <int kMode>
__global__ void __launch_bounds__(512) gather(uint32_t *sink, const uint16_t *src, uint32_t seed) {
  __shared__ uint16_t tab[8192];
  for (int i = threadIdx.x; i < 8192; i += blockDim.x) tab[i] = src[i];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t salt = src[threadIdx.x & 8191u] * 3u + lane * 131u;
  uint32_t acc[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) acc[c] = (seed + c * 977u + lane * 29u) & 8191u;
  const bool on = (src[(lane * 37u) & 8191u] % 100u) < 18u;  // ~18 % of lanes (mode 2)
  const uint32_t vtab = src[lane * 7u];
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
      const uint32_t i = (acc[c] + salt) & 8191u;
      if (kMode == 0) acc[c] = tab[i];
      if (kMode == 1) {
        if (on) acc[c] = tab[i];
        else acc[c] = i;
      }
      if (kMode == 2) acc[c] = tab[(i & ~63u) | lane];
      if (kMode == 3) acc[c] = tab[__builtin_amdgcn_readfirstlane(i)] + lane;
      if (kMode == 4) acc[c] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(i << 2), (int)(vtab + i)) & 0xFFFFu;
      if (kMode == 5) acc[c] = reinterpret_cast<const uint32_t *>(tab)[i & 4095u] & 0xFFFFu;
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) r += acc[c];
  if (r == seed) sink[threadIdx.x] = r;
}

template <int kMode>
float run(int grid, int wg, uint32_t *sink, const uint16_t *src) {
  hipLaunchKernelGGL(gather<kMode>, dim3(grid), dim3(wg * 64), 0, 0, sink, src, 7u);
  (void)hipDeviceSynchronize();
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(gather<kMode>, dim3(grid), dim3(wg * 64), 0, 0, sink, src, 7u);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  uint32_t *sink;
  (void)hipMalloc(&sink, 4096);
  static uint16_t h[8192];
  uint32_t st = 12345u;
  for (int i = 0; i < 8192; ++i) {
    st = st * 1664525u + 1013904223u;
    h[i] = (uint16_t)(st >> 16);
  }
  uint16_t *src;
  (void)hipMalloc(&src, sizeof(h));
  (void)hipMemcpy(src, h, sizeof(h), hipMemcpyHostToDevice);
  const char *names[6] = {"ds_read_u16 random", "ds_read_u16 random, 18% lanes", "ds_read_u16 lane-linear",
                          "ds_read_u16 broadcast", "ds_bpermute_b32", "ds_read_b32 random"};
  for (int wpc : {8, 16, 24}) {
    const int wg = 8;
    const int grid = cus * wpc / wg;
    for (int m = 0; m < 6; ++m) {
      float ms = 0;
      switch (m) {
        case 0: ms = run<0>(grid, wg, sink, src); break;
        case 1: ms = run<1>(grid, wg, sink, src); break;
        case 2: ms = run<2>(grid, wg, sink, src); break;
        case 3: ms = run<3>(grid, wg, sink, src); break;
        case 4: ms = run<4>(grid, wg, sink, src); break;
        default: ms = run<5>(grid, wg, sink, src); break;
      }
      const double per = ms * 1e6 / ((double)kIters * kChains * wpc);  // ns per wave-instruction per CU
      printf("waves/CU %2d  %-30s %7.3f ms  %.2f cyc per wave-instruction per CU (2.1 GHz)  %s\n", wpc, names[m], ms,
             per * 2.1, hipGetErrorString(hipGetLastError()));
    }
  }
  return 0;
}

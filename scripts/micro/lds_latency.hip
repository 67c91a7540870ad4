// lds_latency.hip -- dependent-chain latency of the decoder's LDS table lookups
// (measurement infrastructure): one wave per CU, ONE pointer-chasing chain per lane
// (index = (previous value + lane salt) & mask, so each step is v_add, v_and and the
// read), timed with s_memtime inside the kernel. Modes: random ds_read_u16 from a
// 32 KB u16 table (the single-frame kernel's 14-bit lookup), random ds_read_b32 from
// a 64 KB u32 table, the same two with one address per wave (broadcast, no bank
// conflicts), random ds_read_u8. Prints clocks per step (median over CUs).
//
//   hipcc --offload-arch=gfx950 -O3 -o lds_latency lds_latency.hip && ./lds_latency
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

constexpr int kSteps = 4096;

template <int kMode>
__global__ void __launch_bounds__(64) chase(unsigned long long *clk, uint32_t *sink, const uint32_t *src) {
  __shared__ uint32_t tab[16384];  // 64 KB
  for (int i = threadIdx.x; i < 16384; i += 64) tab[i] = src[i];
  __syncthreads();
  const uint32_t lane = threadIdx.x;
  const uint32_t salt = lane * 2654435761u;
  uint32_t v = src[lane] & 0x3FFFu;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int s = 0; s < kSteps; ++s) {
    const uint32_t x = v + salt;
    if (kMode == 0) v = reinterpret_cast<const uint16_t *>(tab)[x & 0x3FFFu];          // u16, 32 KB
    if (kMode == 1) v = tab[x & 0x3FFFu];                                              // b32, 64 KB
    if (kMode == 2) v = reinterpret_cast<const uint16_t *>(tab)[__builtin_amdgcn_readfirstlane(x) & 0x3FFFu] + lane;
    if (kMode == 3) v = tab[__builtin_amdgcn_readfirstlane(x) & 0x3FFFu] + lane;
    if (kMode == 4) v = reinterpret_cast<const uint8_t *>(tab)[x & 0x7FFFu];           // u8, 32 KB
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  sink[blockIdx.x * 64 + lane] = v;
  if (lane == 0) clk[blockIdx.x] = t1 - t0;
}

template <int kMode>
double run(const char *name, unsigned long long *dclk, uint32_t *dsink, const uint32_t *dsrc, int nblk) {
  chase<kMode><<<nblk, 64>>>(dclk, dsink, dsrc);  // warm
  chase<kMode><<<nblk, 64>>>(dclk, dsink, dsrc);
  if (hipDeviceSynchronize() != hipSuccess) { printf("fault\n"); exit(1); }
  std::vector<unsigned long long> c(nblk);
  hipMemcpy(c.data(), dclk, nblk * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  std::sort(c.begin(), c.end());
  const double med = (double)c[nblk / 2] / kSteps;
  printf("%-28s %6.1f clocks per dependent step (median over %d waves)\n", name, med, nblk);
  return med;
}

int main() {
  const int nblk = 256;  // one wave per CU
  std::vector<uint32_t> h(16384);
  uint32_t s = 12345u;
  for (auto &x : h) { s = s * 1664525u + 1013904223u; x = s >> 8; }
  uint32_t *dsrc, *dsink;
  unsigned long long *dclk;
  hipMalloc(&dsrc, h.size() * 4);
  hipMalloc(&dsink, nblk * 64 * 4);
  hipMalloc(&dclk, nblk * 8);
  hipMemcpy(dsrc, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep) {
    run<0>("ds_read_u16 random", dclk, dsink, dsrc, nblk);
    run<1>("ds_read_b32 random", dclk, dsink, dsrc, nblk);
    run<2>("ds_read_u16 broadcast", dclk, dsink, dsrc, nblk);
    run<3>("ds_read_b32 broadcast", dclk, dsink, dsrc, nblk);
    run<4>("ds_read_u8 random", dclk, dsink, dsrc, nblk);
  }
  return 0;
}

// hbm_sweep.hip -- how high can a plain streaming kernel push HBM on this box? (diagnostic)
// Copy and the decoder's 2:3 read:write mix, 16-B vectors, non-temporal loads/stores,
// U vectors per stream per thread per iteration, grids of G workgroups per CU.
//   hipcc --offload-arch=gfx950 -O3 -o hbm_sweep hbm_sweep.hip && ./hbm_sweep
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int kMix, int U>
__global__ void __launch_bounds__(256) k(const v4u *__restrict__ a, const v4u *__restrict__ b, v4u *__restrict__ d0,
                                         v4u *__restrict__ d1, v4u *__restrict__ d2, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x * U;
  for (size_t base = ((size_t)blockIdx.x * blockDim.x) * U + threadIdx.x; base < n; base += stride) {
    v4u x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + (size_t)u * blockDim.x;
      if (i < n) {
        x[u] = __builtin_nontemporal_load(&a[i]);
        if (kMix) y[u] = __builtin_nontemporal_load(&b[i]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + (size_t)u * blockDim.x;
      if (i < n) {
        __builtin_nontemporal_store(x[u], &d0[i]);
        if (kMix) {
          __builtin_nontemporal_store(y[u], &d1[i]);
          __builtin_nontemporal_store(x[u] ^ y[u], &d2[i]);
        }
      }
    }
  }
}

template <int kMix, int U>
double run(void *a, void *b, void *c, void *d, void *e, size_t n, int grid) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int r = 0; r < 6; ++r) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((k<kMix, U>), dim3(grid), dim3(256), 0, 0, (const v4u *)a, (const v4u *)b, (v4u *)c,
                       (v4u *)d, (v4u *)e, n);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (r && ms < best) best = ms;
  }
  const double bytes = (double)n * 16 * (kMix ? 5 : 2);
  return bytes / (best * 1e-3) / 1e9;
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const size_t n = (size_t)1 << 26;  // 1 GiB per stream
  void *p[5];
  for (int i = 0; i < 5; ++i) {
    (void)hipMalloc(&p[i], n * 16);
    (void)hipMemset(p[i], i, n * 16);
  }
  for (int g : {2, 4, 8, 16, 32}) {
    const int grid = cus * g;
    printf("WG/CU %2d  copy U1 %6.0f U4 %6.0f  |  mix U1 %6.0f U2 %6.0f U4 %6.0f GB/s\n", g,
           run<0, 1>(p[0], p[1], p[2], p[3], p[4], n, grid), run<0, 4>(p[0], p[1], p[2], p[3], p[4], n, grid),
           run<1, 1>(p[0], p[1], p[2], p[3], p[4], n, grid), run<1, 2>(p[0], p[1], p[2], p[3], p[4], n, grid),
           run<1, 4>(p[0], p[1], p[2], p[3], p[4], n, grid));
  }
  return 0;
}

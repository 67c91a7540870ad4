// Micro-benchmark (diagnostic): issue rate of v_lshrrev_b64 vs v_alignbit_b32 vs
// v_add_u32 on gfx950, 8 independent chains per lane, wave64, one workgroup per CU.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int kOp>
__global__ void __launch_bounds__(256) k(unsigned *out, unsigned s, int iters) {
  unsigned a[8], b[8];
  for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x + i; b[i] = threadIdx.x * 3 + i; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (kOp == 0) {
        unsigned long long x = ((unsigned long long)b[i] << 32) | a[i];
        asm volatile("v_lshrrev_b64 %0, %1, %0" : "+v"(x) : "v"(s));
        a[i] = (unsigned)x; b[i] = (unsigned)(x >> 32);
      } else if (kOp == 1) {
        asm volatile("v_alignbit_b32 %0, %1, %0, %2" : "+v"(a[i]) : "v"(b[i]), "v"(s));
      } else {
        asm volatile("v_add_u32 %0, %1, %0" : "+v"(a[i]) : "v"(b[i]));
      }
    }
  }
  unsigned r = 0;
  for (int i = 0; i < 8; ++i) r += a[i] + b[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int kOp>
float run(unsigned *d, int iters, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k<kOp>, dim3(blocks), dim3(256), 0, 0, d, 3u, iters);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<kOp>, dim3(blocks), dim3(256), 0, 0, d, 3u, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  unsigned *d; hipMalloc(&d, (size_t)cus * 4 * 256 * 4);
  const int iters = 20000, blocks = cus * 4;  // 4 waves per SIMD... 16 waves per CU
  const double ops = (double)blocks * 4 /*waves*/ * iters * 8;  // wave-instructions
  const char *names[3] = {"v_lshrrev_b64", "v_alignbit_b32", "v_add_u32"};
  float ms[3] = {run<0>(d, iters, blocks), run<1>(d, iters, blocks), run<2>(d, iters, blocks)};
  for (int i = 0; i < 3; ++i)
    printf("%-16s %8.3f ms  %.2f cycles/wave-instr per SIMD at 2.4 GHz\n", names[i], ms[i],
           ms[i] * 1e-3 * 2.4e9 / (ops / (cus * 4)));
  return 0;
}

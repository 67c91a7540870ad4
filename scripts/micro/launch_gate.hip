// launch_gate.hip -- bench.py's timed-region gate (measurement infrastructure, not
// part of the decoder). The K timed launches are enqueued behind a one-wave kernel
// that polls a host-mapped flag; the clock starts when the host sets the flag. Every
// timed decode still runs inside the timed region -- only the host's enqueue latency
// (graph launch API + doorbell, ~20 us measured at 20 steps) moves before it.
//
// The poll ends by itself after `max_us` (no flag: the gate opens late, never hangs).
// Built by metalhuffman_amd.build.build_probe() into scripts/micro/liblaunch_gate.so.
#include <hip/hip_runtime.h>

#include <stdint.h>

namespace {

__global__ void __launch_bounds__(64) gate_kernel(const unsigned *flag, unsigned long long max_ticks) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz counter
  // system-scope atomic loads: vector memory reads of the host-mapped word
  while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == 0u) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > max_ticks) break;
    __builtin_amdgcn_s_sleep(2);
  }
}

// Tight variant (A/B): relaxed system-scope loads (no cache invalidate per poll), no sleep.
__global__ void __launch_bounds__(64) gate_tight_kernel(const unsigned *flag, unsigned long long max_ticks) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u)
    if (__builtin_amdgcn_s_memrealtime() - t0 > max_ticks) break;
}

// Busy variant (A/B): every workgroup keeps its CU issuing ALU work while the gate is
// closed (so the clocks do not settle down during the host's enqueue); workgroup 0's
// first lane polls the host flag and raises a device flag the others watch.
__global__ void __launch_bounds__(64) gate_busy_kernel(const unsigned *flag, unsigned *dflag,
                                                       unsigned long long max_ticks, float *sink) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  float x = (float)threadIdx.x, y = 1.0001f;
  for (;;) {
    unsigned open;
    if (blockIdx.x == 0) {
      open = __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      if (open && threadIdx.x == 0) __hip_atomic_store(dflag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      open = __hip_atomic_load(dflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (__builtin_amdgcn_readfirstlane(open) || __builtin_amdgcn_s_memrealtime() - t0 > max_ticks) break;
#pragma unroll
    for (int k = 0; k < 64; ++k) x = __builtin_fmaf(x, y, 0.5f);
  }
  if (x == 12345.0f) sink[threadIdx.x] = x;  // keeps the ALU loop
}

}  // namespace

extern "C" {

int gate_arm_tight(unsigned *host_ptr, const unsigned *dev_ptr, void *stream, unsigned max_us) {
  __atomic_store_n(host_ptr, 0u, __ATOMIC_SEQ_CST);
  hipLaunchKernelGGL(gate_tight_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, dev_ptr,
                     (unsigned long long)max_us * 100ull);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Busy gate on `stream`: `nwg` one-wave workgroups; dflag is a device word (cleared here).
int gate_arm_busy(unsigned *host_ptr, const unsigned *dev_ptr, unsigned *dflag, void *stream, unsigned max_us,
                  unsigned nwg, float *sink) {
  __atomic_store_n(host_ptr, 0u, __ATOMIC_SEQ_CST);
  if (hipMemsetAsync(dflag, 0, 4, (hipStream_t)stream) != hipSuccess) return -1;
  hipLaunchKernelGGL(gate_busy_kernel, dim3(nwg), dim3(64), 0, (hipStream_t)stream, dev_ptr, dflag,
                     (unsigned long long)max_us * 100ull, sink);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// A host-mapped, coherent flag word; *host_ptr is written by the host, the kernel
// polls *dev_ptr.
int gate_create(unsigned **host_ptr, unsigned **dev_ptr) {
  void *h = nullptr;
  if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return -1;
  void *d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
    (void)hipHostFree(h);
    return -1;
  }
  *reinterpret_cast<volatile unsigned *>(h) = 0u;
  *host_ptr = static_cast<unsigned *>(h);
  *dev_ptr = static_cast<unsigned *>(d);
  return 0;
}

// Close the flag and enqueue the gate on `stream`; later work on it waits behind.
int gate_arm(unsigned *host_ptr, const unsigned *dev_ptr, void *stream, unsigned max_us) {
  __atomic_store_n(host_ptr, 0u, __ATOMIC_SEQ_CST);
  hipLaunchKernelGGL(gate_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, dev_ptr,
                     (unsigned long long)max_us * 100ull);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The same gate as a stream wait on the flag (hipStreamWaitValue32: the command
// processor itself waits for the value; no kernel). A/B against the polling kernel.
int gate_arm_wait(unsigned *host_ptr, const unsigned *dev_ptr, void *stream) {
  __atomic_store_n(host_ptr, 0u, __ATOMIC_SEQ_CST);
  return hipStreamWaitValue32((hipStream_t)stream, const_cast<unsigned *>(dev_ptr), 1u, hipStreamWaitValueGte,
                              0xFFFFFFFFu) == hipSuccess
             ? 0
             : -1;
}

void gate_open(unsigned *host_ptr) { __atomic_store_n(host_ptr, 1u, __ATOMIC_SEQ_CST); }

void gate_destroy(unsigned *host_ptr) { (void)hipHostFree(host_ptr); }

}  // extern "C"

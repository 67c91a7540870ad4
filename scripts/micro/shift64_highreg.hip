// Minimal reproducer (round 6 forensics, DESIGN.md section 4 "Round 5's miscompute"):
// a 64-bit VALU shift (v_lshrrev_b64) whose shift-amount operand is the LAST VGPR of the
// wave's allocation (v79 with 80 VGPRs allocated) returns a wrong result on gfx950 now
// and then. LLVM works around this hardware bug for gfx90a only
// (GCNHazardRecognizer::fixShift64HighRegBug, "hasShift64HighRegBug": gfx90a, not gfx940+),
// so hipcc for gfx950 emits the pattern unguarded. Round 5's spilled batch-kernel build
// (80 VGPRs) put the step-5 shift amount of its flat-table loop in v79 -- its only 64-bit
// shift with the amount there -- and decoded exactly that symbol wrongly in ~0.5 % of tiles.
//
// Variants (every kernel has the same body; only the registers differ):
//   0  amount in v79, 80 VGPRs allocated (v79 is the last allocated VGPR)      <- suspect
//   1  amount in v78, 80 VGPRs allocated                                         control
//   2  amount in v79, 88 VGPRs allocated (v80..v87 in use)                       control
//   3  amount in v71, 72 VGPRs allocated (the last VGPR of a 72-VGPR wave)       <- suspect
//   4  as 0 with two s_nop between the write of the amount and the shift        (forwarding?)
//   5  amount written into v79 by an SDWA add (src1 WORD_0), 80 VGPRs, shift right after
//      -- the exact pair round 5's build ran at the failing step                 <- suspect
//   6  as 5 into v78 (80 VGPRs)                                                  control
//   7  as 5 with 88 VGPRs                                                        control
//   8  as 5, the SDWA's word operand fresh from an LDS read (ds_read_u16, lgkmcnt(0))
// Each lane shifts a lane- and iteration-dependent 64-bit value by a varying amount and
// counts results that differ from the same shift done in C (v_lshrrev_b64 on low VGPRs).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/micro/shift64_highreg scripts/micro/shift64_highreg.hip
// Run:   scripts/micro/shift64_highreg [launches]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

template <int kVariant>
__device__ __forceinline__ uint64_t shift_hi(uint32_t lo, uint32_t hi, uint32_t amt) {
  uint32_t rlo, rhi;
  if constexpr (kVariant == 0) {
    asm volatile(
        "v_mov_b32 v76, %[lo]\n\tv_mov_b32 v77, %[hi]\n\tv_mov_b32 v79, %[amt]\n\t"
        "v_lshrrev_b64 v[74:75], v79, v[76:77]\n\t"
        "v_mov_b32 %[rlo], v74\n\tv_mov_b32 %[rhi], v75\n\tv_mov_b32 v79, 0\n\t"
        : [rlo] "=v"(rlo), [rhi] "=v"(rhi)
        : [lo] "v"(lo), [hi] "v"(hi), [amt] "v"(amt)
        : "v74", "v75", "v76", "v77", "v79");
  } else if constexpr (kVariant == 1) {
    asm volatile(
        "v_mov_b32 v76, %[lo]\n\tv_mov_b32 v77, %[hi]\n\tv_mov_b32 v78, %[amt]\n\t"
        "v_lshrrev_b64 v[74:75], v78, v[76:77]\n\t"
        "v_mov_b32 %[rlo], v74\n\tv_mov_b32 %[rhi], v75\n\tv_mov_b32 v79, 0\n\t"
        : [rlo] "=v"(rlo), [rhi] "=v"(rhi)
        : [lo] "v"(lo), [hi] "v"(hi), [amt] "v"(amt)
        : "v74", "v75", "v76", "v77", "v78", "v79");
  } else if constexpr (kVariant == 2) {
    asm volatile(
        "v_mov_b32 v76, %[lo]\n\tv_mov_b32 v77, %[hi]\n\tv_mov_b32 v79, %[amt]\n\t"
        "v_mov_b32 v80, %[hi]\n\tv_mov_b32 v87, %[lo]\n\t"
        "v_lshrrev_b64 v[74:75], v79, v[76:77]\n\t"
        "v_mov_b32 %[rlo], v74\n\tv_mov_b32 %[rhi], v75\n\tv_mov_b32 v79, 0\n\t"
        : [rlo] "=v"(rlo), [rhi] "=v"(rhi)
        : [lo] "v"(lo), [hi] "v"(hi), [amt] "v"(amt)
        : "v74", "v75", "v76", "v77", "v79", "v80", "v87");
  } else if constexpr (kVariant == 3) {
    asm volatile(
        "v_mov_b32 v68, %[lo]\n\tv_mov_b32 v69, %[hi]\n\tv_mov_b32 v71, %[amt]\n\t"
        "v_lshrrev_b64 v[66:67], v71, v[68:69]\n\t"
        "v_mov_b32 %[rlo], v66\n\tv_mov_b32 %[rhi], v67\n\tv_mov_b32 v71, 0\n\t"
        : [rlo] "=v"(rlo), [rhi] "=v"(rhi)
        : [lo] "v"(lo), [hi] "v"(hi), [amt] "v"(amt)
        : "v66", "v67", "v68", "v69", "v71");
  } else if constexpr (kVariant == 5 || kVariant == 6 || kVariant == 7) {
    // amt = base + (word & 0xFFFF) with base = amt - 0x1000, word = 0xABCD1000
    const uint32_t base = amt - 0x1000u, word = 0xABCD1000u;
    if constexpr (kVariant == 5)
      asm volatile(
          "v_mov_b32 v76, %[lo]\n\tv_mov_b32 v77, %[hi]\n\t"
          "v_add_u32_sdwa v79, %[b], %[w] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
          "v_lshrrev_b64 v[74:75], v79, v[76:77]\n\t"
          "v_mov_b32 %[rlo], v74\n\tv_mov_b32 %[rhi], v75\n\tv_mov_b32 v79, 0\n\t"
          : [rlo] "=v"(rlo), [rhi] "=v"(rhi)
          : [lo] "v"(lo), [hi] "v"(hi), [b] "v"(base), [w] "v"(word)
          : "v74", "v75", "v76", "v77", "v79");
    else if constexpr (kVariant == 6)
      asm volatile(
          "v_mov_b32 v76, %[lo]\n\tv_mov_b32 v77, %[hi]\n\t"
          "v_add_u32_sdwa v78, %[b], %[w] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
          "v_lshrrev_b64 v[74:75], v78, v[76:77]\n\t"
          "v_mov_b32 %[rlo], v74\n\tv_mov_b32 %[rhi], v75\n\tv_mov_b32 v79, 0\n\t"
          : [rlo] "=v"(rlo), [rhi] "=v"(rhi)
          : [lo] "v"(lo), [hi] "v"(hi), [b] "v"(base), [w] "v"(word)
          : "v74", "v75", "v76", "v77", "v78", "v79");
    else
      asm volatile(
          "v_mov_b32 v76, %[lo]\n\tv_mov_b32 v77, %[hi]\n\tv_mov_b32 v80, %[hi]\n\tv_mov_b32 v87, %[lo]\n\t"
          "v_add_u32_sdwa v79, %[b], %[w] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
          "v_lshrrev_b64 v[74:75], v79, v[76:77]\n\t"
          "v_mov_b32 %[rlo], v74\n\tv_mov_b32 %[rhi], v75\n\tv_mov_b32 v79, 0\n\t"
          : [rlo] "=v"(rlo), [rhi] "=v"(rhi)
          : [lo] "v"(lo), [hi] "v"(hi), [b] "v"(base), [w] "v"(word)
          : "v74", "v75", "v76", "v77", "v79", "v80", "v87");
  } else if constexpr (kVariant == 8) {
    // the word operand from LDS: s_tab[(amt & 63)] holds (amt & 63) + 0x5A5A0000 - base's part
    extern __shared__ uint16_t s_tab[];
    const uint32_t base = amt - (amt & 63u);  // = 0
    const uint32_t addr = (uint32_t)(uintptr_t)(&s_tab[amt & 63u]);
    asm volatile(
        "v_mov_b32 v76, %[lo]\n\tv_mov_b32 v77, %[hi]\n\t"
        "ds_read_u16 v72, %[a]\n\ts_waitcnt lgkmcnt(0)\n\t"
        "v_add_u32_sdwa v79, %[b], v72 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_lshrrev_b64 v[74:75], v79, v[76:77]\n\t"
        "v_mov_b32 %[rlo], v74\n\tv_mov_b32 %[rhi], v75\n\tv_mov_b32 v79, 0\n\t"
        : [rlo] "=v"(rlo), [rhi] "=v"(rhi)
        : [lo] "v"(lo), [hi] "v"(hi), [b] "v"(base), [a] "v"(addr)
        : "v72", "v74", "v75", "v76", "v77", "v79", "memory");
  } else {
    asm volatile(
        "v_mov_b32 v76, %[lo]\n\tv_mov_b32 v77, %[hi]\n\tv_mov_b32 v79, %[amt]\n\t"
        "s_nop 1\n\ts_nop 1\n\t"
        "v_lshrrev_b64 v[74:75], v79, v[76:77]\n\t"
        "v_mov_b32 %[rlo], v74\n\tv_mov_b32 %[rhi], v75\n\tv_mov_b32 v79, 0\n\t"
        : [rlo] "=v"(rlo), [rhi] "=v"(rhi)
        : [lo] "v"(lo), [hi] "v"(hi), [amt] "v"(amt)
        : "v74", "v75", "v76", "v77", "v79");
  }
  return ((uint64_t)rhi << 32) | rlo;
}

template <int kVariant>
__global__ void __launch_bounds__(256) probe(unsigned long long *bad, uint32_t *first, uint32_t seed, int iters) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (kVariant == 8) {
    extern __shared__ uint16_t s_tab[];
    if (threadIdx.x < 64) s_tab[threadIdx.x] = (uint16_t)(threadIdx.x | 0x5A00u);  // low 6 bits = index
    __syncthreads();
  }
  uint32_t s = mix(gid ^ seed);
  unsigned long long nbad = 0;
  for (int i = 0; i < iters; ++i) {
    const uint32_t lo = mix(s + 1u), hi = mix(s + 2u), amt = mix(s + 3u) & 63u;
    s = mix(s);
    const uint64_t want = ((((uint64_t)hi) << 32) | lo) >> amt;
    const uint64_t got = shift_hi<kVariant>(lo, hi, amt);
    if (got != want) {
      ++nbad;
      if (atomicCAS(first, 0u, 1u) == 0u) {  // first mismatch: record amount, want, got
        first[1] = amt;
        first[2] = (uint32_t)want;
        first[3] = (uint32_t)(want >> 32);
        first[4] = (uint32_t)got;
        first[5] = (uint32_t)(got >> 32);
      }
    }
  }
  if (nbad) atomicAdd(bad, nbad);
}

template <int kVariant>
void run(const char *name, int launches, unsigned long long *d_bad, uint32_t *d_first) {
  CHECK(hipMemset(d_bad, 0, sizeof(unsigned long long)));
  CHECK(hipMemset(d_first, 0, 8 * sizeof(uint32_t)));
  const int blocks = 256 * 8, iters = 256;
  for (int l = 0; l < launches; ++l)
    hipLaunchKernelGGL(probe<kVariant>, dim3(blocks), dim3(256), kVariant == 8 ? 128 : 0, 0, d_bad, d_first, 0x9e3779b9u * (l + 1), iters);
  CHECK(hipDeviceSynchronize());
  unsigned long long nbad = 0;
  uint32_t first[8];
  CHECK(hipMemcpy(&nbad, d_bad, sizeof(nbad), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(first, d_first, sizeof(first), hipMemcpyDeviceToHost));
  const double total = (double)launches * blocks * 256 * iters;
  printf("variant %d %-44s shifts %.3e wrong %llu", kVariant, name, total, nbad);
  if (nbad)
    printf("  first: amt %u want %08x%08x got %08x%08x", first[1], first[3], first[2], first[5], first[4]);
  printf("\n");
  fflush(stdout);
}

int main(int argc, char **argv) {
  const int launches = argc > 1 ? atoi(argv[1]) : 20;
  unsigned long long *d_bad;
  uint32_t *d_first;
  CHECK(hipMalloc(&d_bad, sizeof(unsigned long long)));
  CHECK(hipMalloc(&d_first, 8 * sizeof(uint32_t)));
  for (int rep = 0; rep < 2; ++rep) {
    run<0>("amount in v79, 80 VGPRs (last allocated)", launches, d_bad, d_first);
    run<1>("amount in v78, 80 VGPRs", launches, d_bad, d_first);
    run<2>("amount in v79, 88 VGPRs", launches, d_bad, d_first);
    run<3>("amount in v71, 72 VGPRs (last allocated)", launches, d_bad, d_first);
    run<4>("amount in v79, 80 VGPRs, 2 s_nop before", launches, d_bad, d_first);
    run<5>("SDWA add -> v79, 80 VGPRs, shift next", launches, d_bad, d_first);
    run<6>("SDWA add -> v78, 80 VGPRs, shift next", launches, d_bad, d_first);
    run<7>("SDWA add -> v79, 88 VGPRs, shift next", launches, d_bad, d_first);
    run<8>("LDS word -> SDWA add -> v79, 80 VGPRs", launches, d_bad, d_first);
  }
  CHECK(hipFree(d_bad));
  CHECK(hipFree(d_first));
  return 0;
}

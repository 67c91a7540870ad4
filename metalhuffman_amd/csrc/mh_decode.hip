// mh_decode.hip -- CDNA4 (gfx950) Huffman block decoder.
//
// Replaces the reference's per-frame GPU work (Shared/AAPLShaders.metal:127-518 driven
// by Shared/AAPLRenderer.m:1178-1678: 4 x huffFragmentShaderB8W12 + 1 x
// huffFragmentShaderB8W16 render passes, a 16-slice blit and the
// cropAndGrayscaleFromTexturesFragmentShader reorder) with ONE kernel launch that
// writes the W x H 8-bit raster directly.
//
// Work decomposition:
//   * a wavefront owns a "tile" = 64 consecutive 8x8 blocks (one lane per block,
//     block order by*bw + bx as in AAPLShaders.metal:309). For a 2048-wide frame a
//     tile is a 512 x 8 pixel strip whose code bits are one contiguous byte span;
//   * the span is staged into the wave's LDS window with coalesced 16-byte buffer
//     loads, byte-swapped once so the bit cursor reads big-endian dwords;
//   * the lookup table lives in LDS, shared by the workgroup: a 2^13-entry first
//     level and a small second level for the (rare) codes of 14-16 bits. For every
//     16-bit window it returns exactly the {symbol, bitWidth} the reference's T1/T2
//     pair returns (AAPLShaders.metal:159-170), invalid windows included;
//   * each lane runs the 64 serial decode steps of its block from a 64-bit bit
//     window (one LDS word read per two symbols), folds the per-block delta
//     (AAPLShaders.metal:260-262) and stores each finished 8-pixel block row as one
//     8-byte store: the 64 lanes of a wave write 512 contiguous bytes per row.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <stdint.h>

#include <atomic>
#include <mutex>

#include "../../include/metalhuffman.h"
#include "mh_lut.hpp"

namespace {

#ifndef MH_DIAG_STAMPS          // diagnostic builds only: per-wave phase timestamps
#define MH_DIAG_STAMPS 0        //    (scripts/diag_stamps.py)
#endif
#ifndef MH_DIAG_CLOCK           // diagnostic builds only: core-clock cycles of the single-frame
#define MH_DIAG_CLOCK 0         //    decode in stamp slot 5 (scripts/diag_stamps.py --clock)
#endif
#ifndef MH_DIAG_DROP_STORES     // diagnostic builds only: every row store out of range (dropped)
#define MH_DIAG_DROP_STORES 0
#endif
#ifndef MH_LANE_PAIRS           // 1: the lane-pair diagnostic library only (libmh_diag_lanepairs.so,
#define MH_LANE_PAIRS 0         //    metalhuffman_amd/build.py), which exports mh_diag_decode_lanepairs
#endif
constexpr int kStageBytes = 4352;             // per-wave LDS window (max tile span)
constexpr int kMaxWavesPerWG = 8;             // batch kernel workgroup width
constexpr int kMinWavesPerEU = 6;             // register cap: 6 waves/SIMD = what the LDS budget admits
// Row-store cache bits (gfx950 aux field: 1 sc0, 2 nt, 16 sc1). Batch kernel: nt.
// Small-launch kernel: nt sc1, write-through, so nothing dirty is left in the XCDs'
// L2s for the end-of-kernel release to write back (profiles/r03_v5_store_write_through_ab.txt;
// both re-checked cold in round 5: profiles/r05_batch_store_policy_ab.txt, r05_small_store_policy_ab.txt).
constexpr int kBatchStoreAux = 2;
constexpr int kSmallStoreAux = 18;
static_assert(kStageBytes % 16 == 0, "stage uses 16-byte chunks");

typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));

struct DecodeArgs {
  const uint32_t *offsets;     // frame f's block offsets at offsets + f*nb
  const uint8_t *codes;
  const uint64_t *frame_off;   // n_frames+1 entries, or null
  uint64_t codes_bytes;
  const uint16_t *t1;          // HuffLookupSymbol viewed as u16 = symbol | bitWidth << 8
  const uint16_t *t2;
  const uint16_t *lut;         // prepared L1+L2 table or null
  const uint8_t *block_init;
  uint8_t *out;
  uint64_t out_pitch;
  uint64_t out_frame_stride;
  uint64_t out_frame_bytes;    // H * pitch
  uint32_t t2_entries;
  uint32_t w, h, bw, bh, nb;
  uint32_t tiles_per_frame, total_tiles;
  uint32_t n_groups;           // ceil(total_tiles / waves_per_wg)
  uint32_t nwaves, grid;       // batch kernel launch shape as kernel arguments: blockDim / gridDim
                               // read the dispatch packet's implicit arguments, a dependent
                               // global load at the head of the kernel (code object v5)
};

__device__ __forceinline__ uint32_t bswap32(uint32_t x) {
  return __builtin_amdgcn_perm(0u, x, 0x00010203u);
}

// AAPLShaders.metal:159-170 / HuffmanUtil.cpp:961-995 on a 16-bit pattern.
// Out-of-range T2 reads (corrupt tables only) return the all-zero entry.
__device__ __forceinline__ uint32_t split_lookup(const uint16_t *t1, const uint16_t *t2,
                                                 uint32_t t2_entries, uint32_t pat16) {
  uint32_t e = t1[pat16 >> 8];
  if ((e >> 8) == 0) {
    const uint32_t idx = (e & 0xFFu) * 256u + (pat16 & 0xFFu);
    e = idx < t2_entries ? (uint32_t)t2[idx] : 0u;
  }
  return e;
}


// Builds the two-level table into `lut` (LDS or global) with `nthreads`
// cooperating threads; `p0` is a scratch word shared by them.
//   L1[p] (p = 13-bit prefix): step_word(split_lookup(p << 3)) when that code has
//     <= 13 bits or the window is invalid (0 -> no-op, as the reference's dummy
//     T2 subtable, HuffmanUtil.cpp:550-556); otherwise an escape `sub`.
//     Canonical codes are ordered by length, so every code of 14-16 bits lies at
//     or above the first such code's prefix P0 and the long codes (<= 256 codes
//     of >= 4 patterns) occupy at most 128 prefixes from P0.
//   L2[sub*8 + x] = step_word(split_lookup(((P0 + sub - 1) << 3) | x)), sub >= 1;
//   L2 subtable 0 is all zero (escapes beyond the long-code range: invalid windows).
template <class SyncFn>
__device__ void build_lut(const uint16_t *t1, const uint16_t *t2, uint32_t t2_entries,
                          uint16_t *lut, uint32_t *p0, uint32_t tid, uint32_t nthreads,
                          SyncFn sync) {
  if (tid == 0) *p0 = (uint32_t)kL1Entries;
  sync();
  for (uint32_t p = tid; p < (uint32_t)kL1Entries; p += nthreads) {
    const uint32_t e = split_lookup(t1, t2, t2_entries, p << kL2Bits);
    lut[p] = (uint16_t)step_word(e);
    if ((e >> 8) > (uint32_t)kLutBits) atomicMin(p0, p);
  }
  for (uint32_t i = tid; i < (uint32_t)(kLutEntries - kL1Entries); i += nthreads)
    lut[kL1Entries + i] = 0;
  sync();
  const uint32_t P0 = *p0;
  for (uint32_t p = P0 + tid; p < (uint32_t)kL1Entries; p += nthreads) {
    const uint32_t sub = p - P0 + 1;
    lut[p] = (uint16_t)(sub < (uint32_t)kL2Subtables ? sub : 0u);
  }
  const uint32_t nl2 = ((uint32_t)kL1Entries - P0) << kL2Bits;
  for (uint32_t i = tid; i < nl2 && i < (uint32_t)(kL2Entries - (1 << kL2Bits)); i += nthreads)
    lut[kL1Entries + (1 << kL2Bits) + i] =
        (uint16_t)step_word(split_lookup(t1, t2, t2_entries, (P0 << kL2Bits) + i));
  sync();
}


#if !MH_LANE_PAIRS
// mh_prepare_lut: the prepared tables from T1/T2 in device memory, one workgroup
// (build_prepared_lut, mh_lut.hpp).
__global__ void __launch_bounds__(1024) mh_prepare_lut_kernel(const uint16_t *t1, const uint16_t *t2,
                                                              uint32_t t2_entries, uint8_t *buf) {
  __shared__ uint16_t s_t1[256];
  __shared__ uint32_t s_scratch[4];
  if (threadIdx.x < 256) s_t1[threadIdx.x] = t1[threadIdx.x];
  __syncthreads();
  build_prepared_lut(s_t1, t2, t2_entries, buf, s_scratch);
}
#endif

// Word source for the bit cursor: big-endian dwords of the tile's code span.
struct LdsWords {
  const uint8_t *w;
  __device__ __forceinline__ const uint8_t *at(uint32_t byte_off) const { return w + byte_off; }
};
// Stage swizzle (batch kernel, flat tables only): the eight 16-B chunks of every
// 128-B row of a wave's stage are permuted by the row index (XOR), so lanes whose
// blocks start a multiple of 128 B apart -- flat code lengths make every block
// exactly 64 B -- refill from different LDS banks (b32 reads bank on (a/4) mod 32).
// Chunks stay whole (16-B staging stores) and stay inside their row.
__device__ __forceinline__ uint32_t swz_off(uint32_t o) { return o ^ ((o >> 3) & 0x70u); }

// byte 1 (prev) of four successive lane states -> one output word, 3 VALU
__device__ __forceinline__ uint32_t pack_prev4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  const uint32_t lo = __builtin_amdgcn_perm(b, a, 0x0C0C0501u);  // [a.1, b.1, 0, 0]
  const uint32_t hi = __builtin_amdgcn_perm(d, c, 0x05010C0Cu);  // [0, 0, c.1, d.1]
  return lo | hi;
}

// byte 0 of four successive sums -> one output word, 3 VALU
__device__ __forceinline__ uint32_t pack_lo4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  const uint32_t lo = __builtin_amdgcn_perm(b, a, 0x0C0C0400u);  // [a.0, b.0, 0, 0]
  const uint32_t hi = __builtin_amdgcn_perm(d, c, 0x04000C0Cu);  // [0, 0, c.0, d.0]
  return lo | hi;
}

// v_perm_b32 selectors: put S0.byte1 at byte J, keep S1's other bytes
__device__ __forceinline__ constexpr uint32_t ins_sel1(int j) {
  return j == 0 ? 0x03020105u : j == 1 ? 0x03020500u : j == 2 ? 0x03050100u : 0x05020100u;
}

__shared__ __attribute__((aligned(16))) uint16_t s_lut[kLutEntries];
__shared__ __attribute__((aligned(16))) uint8_t s_stage[kMaxWavesPerWG * kStageBytes];
__shared__ uint32_t s_p0;

#if MH_DIAG_STAMPS
constexpr int kDiagWaves = 8192, kDiagSlots = 8;
__device__ unsigned long long g_stamps[kDiagWaves * kDiagSlots];
#define MH_STAMP(i) (ts[i] = __builtin_amdgcn_s_memrealtime())
#else
#define MH_STAMP(i) ((void)0)
#endif

// Wave priority 0..3 (s_setprio takes an immediate). The SIMD arbiter serves the
// oldest wave first among equal priorities, so waves of later workgroups fall
// behind; the batch loop gives waves with more tiles left a higher priority.
__device__ __forceinline__ void set_prio(uint32_t p) {
  switch (__builtin_amdgcn_readfirstlane(p) & 3u) {
    case 0: __builtin_amdgcn_s_setprio(0); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3); break;
  }
}

// Lookup flavours of the decode step.
//   Lut13: 2^13-entry first level + escapes to the second level (any code <= 16 bits).
//   Lut14: 2^14-entry single level, no escape test at all; valid when no code is
//          longer than 14 bits (the prepared table records the longest code).
// kMasked: only the lanes that consumed a word read the next one (batch kernel);
//   the small-launch kernel's latency-bound chain reads unmasked.
// kLazy: the refill test runs at every step on the cursor the lookup itself uses, in the
//   lookup's LDS shadow, and takes effect at the next step (the small kernel's step since
//   round 5: profiles/r05_lazy_ab.txt) (sh <= 47 still holds at every
//   lookup: sh >= 32 drops a word, sh < 32 advances by <= 16), so the chain from one
//   lookup to the next is add, shift, and -- no compare / select on it.
template <int kBits, bool kMaskedRefill, bool kEscapes = kBits == kLutBits, bool kSwizzle = false,
          int kStoreAux = kBatchStoreAux, bool kLazyRefill = false, bool kFlat8Bytes = false>
struct StepCfg {
  static constexpr bool kLazy = kLazyRefill;
  static constexpr bool kFlat8 = kFlat8Bytes;  // flat 8-bit canonical table: byte arithmetic
  static constexpr int kAux = kStoreAux;  // row-store cache bits
  static constexpr bool kEsc = kEscapes;
  static constexpr bool kSwz = kSwizzle;
  static constexpr bool kMasked = kMaskedRefill;
  static constexpr uint32_t kCur = 127u - (uint32_t)kBits;   // S low byte = kCur - sh
  static constexpr uint32_t kMask = (2u << kBits) - 2u;       // byte address of a u16 entry
  static constexpr uint32_t kRefillAt = kCur - 32u;           // low byte <= this: sh >= 32
};

using Lut13 = StepCfg<kLutBits, true>;  // the batch kernel's step
// ... and its escape-free twin, for tables whose longest code is <= 13 bits (the
// first level then decodes every window; no per-symbol escape test)
using Lut13NoEsc = StepCfg<kLutBits, true, false>;
// ... and for flat tables (every code the same length, e.g. uniform bytes: every
// block the same size, so lanes sit a multiple of 128 B apart): swizzled stage
using Lut13Flat = StepCfg<kLutBits, true, false, true>;

// One lane decodes one 8x8 block: 64 serial steps of AAPLShaders.metal:241-268
// (cursor advance + delta fold); each finished 8-pixel block row is stored at once.
//
// Lane state: a 64-bit window hi:lo of big-endian code words, the LDS address
// `wa` of hi in the staged span, the prefetched next word `nw`, and
//   S: bits 0-7 = kCur - sh (sh = bits of hi:lo already consumed, 0..63),
//      bits 8-15 = prev (the running delta sum), bits 16+ = don't care.
// (hi:lo) >> (S & 63) = (hi:lo) >> (kCur - 64 - sh) puts the next kBits code bits
// at bits 1..kBits, i.e. the byte address of their u16 table entry; one add of the
// entry's step word then advances sh and prev together (the low byte stays in
// [kCur - 63, kCur], so it never borrows from prev).
template <bool kDelta, class Cfg, class Src>
__device__ __forceinline__ void decode_block(const Src &src, const uint8_t *lut, uint32_t p,
                                             uint32_t prev, __amdgpu_buffer_rsrc_t out,
                                             uint32_t row0, uint32_t pitch, bool dead) {
  if constexpr (Cfg::kFlat8) {
    // 64 one-byte codes from bit p of the staged (big-endian word) span: 17 words, each
    // output word a 64-bit funnel shift (any bit alignment); code c is symbol c
    typedef const __attribute__((address_space(3))) uint32_t *lds_u32;
    typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));
    const lds_u32 wp = (lds_u32)(src.w + (p >> 5) * 4u);
    const uint32_t sh = p & 31u;
    uint32_t w[17];
#pragma unroll
    for (int j = 0; j < 17; ++j) w[j] = wp[j];
    const uint32_t rbase = dead ? 0x80000000u : row0;
    uint32_t s = prev;
#pragma unroll
    for (uint32_t r = 0; r < 8; ++r) {
      uint32_t c[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t j = 2 * r + h;
        c[h] = (uint32_t)(((((uint64_t)w[j]) << 32 | w[j + 1]) << sh) >> 32);  // big-endian: symbol 4j+i = byte 3-i
      }
      v2u32 v;
      if (kDelta) {
        uint32_t sv[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
          for (int i = 0; i < 4; ++i) sv[i] = s = s + ((c[h] >> (24 - 8 * i)) & 0xFFu);
          const uint32_t o = pack_lo4(sv[0], sv[1], sv[2], sv[3]);
          if (h) v.y = o; else v.x = o;
        }
      } else {
        v.x = bswap32(c[0]);
        v.y = bswap32(c[1]);
      }
      __builtin_amdgcn_raw_buffer_store_b64(v, out, (int)(rbase + r * pitch), 0, Cfg::kAux);
    }
    return;
  }
  // wa: LDS address of hi's word in the staged span. An explicit local-address-space
  // pointer keeps its arithmetic 32-bit (a generic pointer was carried as a 64-bit value:
  // one 64-bit add per refill) and lets the reads fold their constant offsets.
  typedef const __attribute__((address_space(3))) uint8_t *lds_u8;
  typedef const __attribute__((address_space(3))) uint32_t *lds_u32;
  const lds_u8 base = (lds_u8)src.w;
  lds_u8 wa = base + (p >> 5) * 4u;
  const auto rd = [&](lds_u8 q) -> uint32_t {
    if constexpr (Cfg::kSwz)
      return *(lds_u32)(base + swz_off((uint32_t)(q - base)));
    else
      return *(lds_u32)q;
  };
  uint32_t S = (prev << 8) + Cfg::kCur - (p & 31u);
  // An odd refill bound (the 14-bit table's) goes in as an opaque scalar: as a literal
  // the compiler rewrites (S & 0xFF) <= K as (S & 0xFE) < K + 1, which no longer folds
  // into a byte-select (SDWA) compare -- one more VALU on every refill step's chain.
  uint32_t kRefill = Cfg::kRefillAt;
  if constexpr ((Cfg::kRefillAt & 1u) != 0u) asm("s_mov_b32 %0, %1" : "=s"(kRefill) : "n"(Cfg::kRefillAt));
  uint32_t hi = rd(wa);
  uint32_t lo = rd(wa + 4);
  uint32_t nw = rd(wa + 8);

  // sh <= 47 at every lookup keeps >= 16 valid window bits.
#define MH_LOOKUP(A1)                                                               \
  uint32_t e = *reinterpret_cast<const uint16_t *>(lut + (A1));
#define MH_FINISH(J, OW)                                                            \
  {                                                                                 \
    if constexpr (Cfg::kEsc) {                                                      \
      const bool esc = e < kEscapeBelow;                                            \
      if (__builtin_expect(__ballot(esc) != 0, 0)) {                                \
        const uint64_t x = (((uint64_t)hi) << 32) | lo;                             \
        const uint32_t x3 = (uint32_t)(x >> ((S - 2u) & 63u)) & 7u;                 \
        const uint32_t e2 = *reinterpret_cast<const uint16_t *>(                    \
            lut + 2u * (kL1Entries + ((e & 0xFFu) << kL2Bits) + x3));               \
        e = esc ? e2 : e;                                                           \
      }                                                                             \
    }                                                                               \
    S += e;                                                                         \
    if (kDelta) {                                                                   \
      sv[J] = S;  /* packed four at a time (pack_prev4) */                         \
    } else {                                                                        \
      OW = __builtin_amdgcn_perm(e + 0xFFu, OW, ins_sel1(J));  /* byte 1: symbol */  \
    }                                                                               \
  }
#define MH_STEP(J, OW)                                                              \
  {                                                                                 \
    const uint64_t x = (((uint64_t)hi) << 32) | lo;                                 \
    MH_LOOKUP((uint32_t)(x >> (S & 63u)) & Cfg::kMask)                              \
    MH_FINISH(J, OW)                                                                \
  }
  // keep sh < 32 at the start of every symbol pair (each code is <= 16 bits)
#define MH_REFILL_C(c)                                                              \
  {                                                                                 \
    hi = c ? lo : hi;                                                               \
    lo = c ? nw : lo;                                                               \
    const uint32_t d = c ? 4u : 0u;                                                 \
    wa += d;                                                                        \
    /* swizzled stage: keep wa one register (else it is re-derived as a sum of */  \
    /* every step's d inside each masked refill, which spills)                */  \
    if constexpr (Cfg::kSwz) asm volatile("" : "+v"(wa));                          \
    /* masked refill: the selects stay selects (v_cndmask) -- else the compiler   */  \
    /* folds them into the masked read's if-block as exec-masked copies (8 moves  */  \
    /* at every row start)                                                        */  \
    if constexpr (Cfg::kMasked) asm volatile("" : "+v"(hi), "+v"(lo));             \
    S += d * 8u;                                                                    \
    if constexpr (!Cfg::kMasked) nw = rd(wa + 8);                                   \
  }
#define MH_STEP_L(J, OW)                                                            \
  {                                                                                 \
    const uint64_t x = (((uint64_t)hi) << 32) | lo;                                 \
    MH_LOOKUP((uint32_t)(x >> (S & 63u)) & Cfg::kMask)                              \
    /* off the chain: refill from the cursor this lookup used */                    \
    const bool c = (S & 0xFFu) <= kRefill;                                         \
    hi = c ? lo : hi;                                                               \
    lo = c ? nw : lo;                                                               \
    const uint32_t d = c ? 4u : 0u;                                                 \
    wa += d;                                                                        \
    S += d * 8u;                                                                    \
    /* keep S + d*8 one add ahead of S + e (else it is re-associated onto the  */  \
    /* chain), and the selects as selects                                       */  \
    asm volatile("" : "+v"(S), "+v"(hi), "+v"(lo));                                \
    /* the next word at even steps only: wa changes only at a refill and no     */  \
    /* refill follows a refill, so an even step lies between two refills and its */ \
    /* read lands a step before the next one needs it (half the stage reads)     */ \
    if constexpr (((J) & 1) == 0) nw = rd(wa + 8);                                 \
    MH_FINISH(J, OW)                                                                \
  }
#define MH_STEP_R(J, OW)                                                            \
  {                                                                                 \
    const bool c = (S & 0xFFu) <= kRefill;                                         \
    MH_REFILL_C(c)                                                                  \
    MH_STEP(J, OW)                                                                  \
    /* masked: only lanes that consumed a word fetch the next (issued behind the */ \
    /* lookup; fewer active lanes -> fewer LDS bank conflicts)                   */ \
    if constexpr (Cfg::kMasked) {                                                   \
      if (c) nw = rd(wa + 8);                                                       \
    }                                                                               \
  }

  // dead lanes store at >= 2^31 + r * pitch: past every output descriptor's range
  // (<= 0x7FFFFFF0 bytes), so the hardware drops them -- one select per tile, not per row
  const uint32_t rbase = (dead || MH_DIAG_DROP_STORES) ? 0x80000000u : row0;
#pragma unroll
  for (uint32_t r = 0; r < 8; ++r) {
    uint32_t o0 = 0, o1 = 0;
    uint32_t sv[4];  // S after each symbol of the current output word (delta mode)
    (void)sv;
    if constexpr (Cfg::kLazy) {
      MH_STEP_L(0, o0);
      MH_STEP_L(1, o0);
      MH_STEP_L(2, o0);
      MH_STEP_L(3, o0);
      if (kDelta) o0 = pack_prev4(sv[0], sv[1], sv[2], sv[3]);
      MH_STEP_L(0, o1);
      MH_STEP_L(1, o1);
      MH_STEP_L(2, o1);
      MH_STEP_L(3, o1);
      if (kDelta) o1 = pack_prev4(sv[0], sv[1], sv[2], sv[3]);
    } else {
    if (r) {
      MH_STEP_R(0, o0);
    } else {
      MH_STEP(0, o0);
    }
    MH_STEP(1, o0);
    MH_STEP_R(2, o0);
    MH_STEP(3, o0);
    if (kDelta) o0 = pack_prev4(sv[0], sv[1], sv[2], sv[3]);
    MH_STEP_R(0, o1);
    MH_STEP(1, o1);
    MH_STEP_R(2, o1);
    MH_STEP(3, o1);
    if (kDelta) o1 = pack_prev4(sv[0], sv[1], sv[2], sv[3]);
    }
    // Unconditional 8-byte row store (exact vmcnt counting): lanes without a
    // block and rows below the frame use offsets outside the descriptor's range,
    // which the hardware drops. A right-edge block writes its 8 bytes into the
    // row's pitch padding (pitch >= round_up(W, 8)).
    {
      typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));
      v2u32 v;
      v.x = o0;
      v.y = o1;
      const uint32_t off = rbase + r * pitch;
      __builtin_amdgcn_raw_buffer_store_b64(v, out, (int)off, 0, Cfg::kAux);
    }
  }
#undef MH_STEP
#undef MH_STEP_R
#undef MH_STEP_L
#undef MH_LOOKUP
#undef MH_FINISH
#undef MH_REFILL_C
}

constexpr int kStageChunks = (kStageBytes / 16 + 63) / 64;  // 16-B chunks per lane (5)

// Buffer descriptors from provably wave-uniform inputs (readfirstlane), so hipcc
// does not wrap each buffer op in a waterfall loop (cdna_hip_programming.md T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void *base, uint32_t bytes) {
  const uint64_t p = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// A tile's header loads (issued one tile ahead; all VMEM so that no scalar load
// is pending in lgkmcnt while the decode waits on LDS reads).
// tile -> frame. A launch of one frame skips the division (a uniform branch): the
// division is ~30 instructions ahead of a wave's first HBM load (its block offsets).
__device__ __forceinline__ uint32_t frame_of(const DecodeArgs &a, uint32_t tile) {
  if (a.total_tiles <= a.tiles_per_frame) return 0u;
  return tile / a.tiles_per_frame;
}

struct TileHdr {
  uint32_t tile;      // wave-uniform; >= total_tiles: no tile
  uint32_t off;       // this lane's block start bit
  uint32_t nxt;       // next block's start bit (this lane's block end)
  uint32_t fo_lo, fo_hi;  // lanes 0/1: frame_off[f], frame_off[f+1]
  uint32_t init;      // per-block initial prev (block_init) or 0
};

__device__ __forceinline__ void hdr_issue(const DecodeArgs &a, uint32_t tile, uint32_t lane,
                                          TileHdr &h) {
  // Branch-free: absent arrays (frame_off / block_init == NULL) get descriptors
  // with zero records, whose loads return 0 without touching memory; a past-the-end
  // tile reads through zero-record descriptors too. Unconditional loads keep the
  // compiler from waiting on the span prefetch to re-zero these registers.
  tile = __builtin_amdgcn_readfirstlane(tile);
  const bool live = tile < a.total_tiles;
  const uint32_t f = live ? frame_of(a, tile) : 0u;
  const uint32_t b = (live ? (tile - f * a.tiles_per_frame) * 64u : 0u) + lane;
  h.tile = tile;
  const __amdgpu_buffer_rsrc_t ro = uniform_rsrc(a.offsets + (uint64_t)f * a.nb, live ? a.nb * 4u : 0u);
  h.off = __builtin_amdgcn_raw_buffer_load_b32(ro, (int)(b * 4u), 0, 0);
  h.nxt = __builtin_amdgcn_raw_buffer_load_b32(ro, (int)(b * 4u + 4u), 0, 0);
  typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));
  const __amdgpu_buffer_rsrc_t rf = uniform_rsrc(
      a.frame_off ? (const void *)a.frame_off : (const void *)a.offsets,
      (live && a.frame_off) ? 0x7FFFFFF0u : 0u);
  const v2u32 v = __builtin_amdgcn_raw_buffer_load_b64(rf, (int)((f + (lane & 1u)) * 8u), 0, 0);
  h.fo_lo = v.x;
  h.fo_hi = v.y;
  const __amdgpu_buffer_rsrc_t ri = uniform_rsrc(
      a.block_init ? (const void *)(a.block_init + (uint64_t)f * a.nb) : (const void *)a.offsets,
      (live && a.block_init) ? a.nb : 0u);
  h.init = __builtin_amdgcn_raw_buffer_load_b8(ri, (int)b, 0, 0);
}

// Everything derived from a header once its loads have landed.
struct Tile {
  uint32_t tile, f, b0;
  bool valid;          // this lane holds a block
  uint32_t p;          // lane's start bit relative to the staged span
  uint32_t start;      // span start byte (16-aligned, frame relative)
  uint32_t span;       // span bytes (0xFFFFFFFF: unknown / corrupt)
  uint32_t fb32;       // frame bytes (clamped to u32)
  uint64_t fbeg;
  uint32_t init;
  uint32_t span_end_bits;  // end bit of the tile's last block (frame relative)
};

__device__ __forceinline__ Tile hdr_resolve(const DecodeArgs &a, const TileHdr &h, uint32_t lane) {
  Tile t;
  t.tile = h.tile;
  t.f = frame_of(a, h.tile);
  t.b0 = (h.tile - t.f * a.tiles_per_frame) * 64u;
  const uint32_t b = t.b0 + lane;
  t.valid = b < a.nb;
  uint64_t fbytes = a.codes_bytes;
  t.fbeg = 0;
  if (a.frame_off) {
    const uint64_t lo = ((uint64_t)__builtin_amdgcn_readlane(h.fo_hi, 0) << 32) |
                        __builtin_amdgcn_readlane(h.fo_lo, 0);
    const uint64_t hi = ((uint64_t)__builtin_amdgcn_readlane(h.fo_hi, 1) << 32) |
                        __builtin_amdgcn_readlane(h.fo_lo, 1);
    t.fbeg = lo;
    fbytes = hi - lo;
  }
  t.fb32 = (uint32_t)(fbytes > 0xFFFFFFF0ull ? 0xFFFFFFF0ull : fbytes);
  const uint32_t fbits = t.fb32 > 0x1FFFFFFFu ? 0xFFFFFFFFu : t.fb32 * 8u;
  // a frame's last block ends at most 64 x 16 bits after its start, whatever the
  // buffer size (a reused streaming slot is larger than the frame it holds)
  const uint32_t end_l = (b + 1u < a.nb) ? h.nxt : min(fbits, h.off + 64u * 16u);
  const uint32_t last = min(63u, a.nb - 1u - t.b0);  // last lane holding a block
  const uint32_t sb = __builtin_amdgcn_readfirstlane(h.off);
  const uint32_t eb = __builtin_amdgcn_readlane(end_l, last);
  t.span_end_bits = eb;
  t.start = (sb >> 3) & ~15u;
  uint32_t end = (eb >> 3) + 24u;
  if (end > t.fb32 + 16u) end = t.fb32 + 16u;
  t.span = end > t.start ? ((end - t.start + 15u) & ~15u) : 0xFFFFFFFFu;
  t.p = t.valid ? h.off - t.start * 8u : 0u;
  t.init = h.init & 0xFFu;
  // materialise every header-derived value now: the loads are a tile old, and no
  // later use may make the compiler wait on the span prefetch issued after this
  asm volatile("" ::"v"(t.p), "v"(t.init));
  return t;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t codes_rsrc(const DecodeArgs &a, const Tile &t) {
  return uniform_rsrc(a.codes + t.fbeg, t.fb32);
}

// Output addressing of a tile: a store descriptor based at the tile's first block
// row (64-bit base, so frames beyond 4 GB of raster work) and each lane's offset
// of its block's first row from there. Stores below row H fall outside the
// descriptor's range and are dropped.
struct OutTile {
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t row0;
};
__device__ __forceinline__ OutTile out_tile(const DecodeArgs &a, const Tile &t, uint32_t lane) {
  const uint32_t b = t.b0 + lane;
  const uint32_t bx = b % a.bw, by = b / a.bw;
  const uint32_t by0 = __builtin_amdgcn_readfirstlane(t.b0 / a.bw);
  const uint64_t base = (uint64_t)by0 * 8u * a.out_pitch;
  const uint64_t rem = a.out_frame_bytes > base ? a.out_frame_bytes - base : 0u;
  OutTile o;
  o.rsrc = uniform_rsrc(a.out + (uint64_t)t.f * a.out_frame_stride + base,
                        (uint32_t)(rem < 0x7FFFFFF0ull ? rem : 0x7FFFFFF0ull));
  o.row0 = (by - by0) * 8u * (uint32_t)a.out_pitch + bx * 8u;
  return o;
}

__device__ __forceinline__ void span_issue(const DecodeArgs &a, const Tile &t, uint32_t lane,
                                           v4u32 (&R)[kStageChunks], bool on = true) {
  // Unconditional loads (no exec-masked branches, so the compiler can count them
  // in vmcnt); chunks past the span use an offset outside the descriptor's range,
  // which returns 0 without a memory access.
  // not `on`: a zero-record descriptor, so no offset can reach memory
  const __amdgpu_buffer_rsrc_t rc = uniform_rsrc(a.codes + (on ? t.fbeg : 0ull), on ? t.fb32 : 0u);
  // one wave-uniform byte count, so the compiler cannot split the loads by `on`
  const uint32_t span = __builtin_amdgcn_readfirstlane(on ? t.span : 0u);
#pragma unroll
  for (int k = 0; k < kStageChunks; ++k) {
    const uint32_t c = lane + 64u * k;
    const uint32_t off = c * 16u < span ? t.start + c * 16u : 0xFFFFFFF0u;
    R[k] = __builtin_amdgcn_raw_buffer_load_b128(rc, (int)off, 0, 0);
  }
}

template <bool kSwz = false>
__device__ __forceinline__ void span_write(const Tile &t, uint32_t lane, const v4u32 (&R)[kStageChunks],
                                           uint8_t *stage) {
#pragma unroll
  for (int k = 0; k < kStageChunks; ++k) {
    const uint32_t c = lane + 64u * k;
    if (c * 16u < t.span) {
      v4u32 v = R[k];
      v.x = bswap32(v.x);
      v.y = bswap32(v.y);
      v.z = bswap32(v.z);
      v.w = bswap32(v.w);
      *reinterpret_cast<v4u32 *>(stage + (kSwz ? swz_off(c * 16u) : c * 16u)) = v;
    }
  }
}

// A workgroup barrier for LDS-only hand-offs: waits for this wave's LDS operations
// (lgkmcnt), not its global ones -- __syncthreads()'s workgroup-scope fence also waits
// for every outstanding global load (vmcnt(0)), here the first header.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Oversize tile: stage + decode lanes [0,32) then [32,64), each from its own span.
template <bool kDelta, class Cfg>
__device__ __forceinline__ void decode_halves(const DecodeArgs &a, const Tile &t, uint32_t lane,
                                              const uint8_t *lut, uint8_t *stage,
                                              __amdgpu_buffer_rsrc_t out, uint32_t row0, bool dead) {
  const __amdgpu_buffer_rsrc_t rc = codes_rsrc(a, t);
  const uint32_t my_off = t.p + t.start * 8u;  // lane's absolute start bit
  const uint32_t fbits = t.fb32 > 0x1FFFFFFFu ? 0xFFFFFFFFu : t.fb32 * 8u;
#pragma unroll 1
  for (uint32_t h = 0; h < 2; ++h) {
    const uint32_t first = h * 32u;
    const uint32_t sb = __builtin_amdgcn_readlane(my_off, first);
    // end of the half: start bit of lane first+32 (or the tile's last block end)
    const uint32_t nblk = a.nb - t.b0;  // blocks in this tile (may be < 64)
    if (first >= nblk) break;
    uint32_t eb;
    if (first + 32u < nblk) {
      eb = __builtin_amdgcn_readlane(my_off, first + 32u);
    } else {
      eb = t.span_end_bits;
    }
    const uint32_t start = (sb >> 3) & ~15u;
    uint32_t end = (eb >> 3) + 24u;
    if (end > t.fb32 + 16u) end = t.fb32 + 16u;
    const uint32_t span = min((end - start + 15u) & ~15u, (uint32_t)kStageBytes);
    __builtin_amdgcn_s_waitcnt(0);  // rare path: drain before reusing the window
    for (uint32_t c = lane; c * 16u < span; c += 64u) {
      v4u32 v = __builtin_amdgcn_raw_buffer_load_b128(rc, (int)(start + c * 16u), 0, 0);
      v.x = bswap32(v.x);
      v.y = bswap32(v.y);
      v.z = bswap32(v.z);
      v.w = bswap32(v.w);
      *reinterpret_cast<v4u32 *>(stage + (Cfg::kSwz ? swz_off(c * 16u) : c * 16u)) = v;
    }
    wave_sync();
    if (lane >= first && lane < first + 32u) {
      LdsWords src{stage};
      decode_block<kDelta, Cfg>(src, lut, t.valid ? my_off - start * 8u : 0u, t.init, out, row0,
                                (uint32_t)a.out_pitch, dead);
    }
    wave_sync();
  }
  __builtin_amdgcn_s_waitcnt(0);
  (void)fbits;
}

#if MH_DIAG_STAMPS
#define MH_TS_PARAM , unsigned long long (&ts)[kDiagSlots]
#define MH_TS_ARG , ts
#else
#define MH_TS_PARAM
#define MH_TS_ARG
#endif

// static grid-stride schedule; a tile id >= total_tiles means "no tile"
__device__ __forceinline__ uint32_t next_tile(const DecodeArgs &a, uint32_t t, uint32_t gstride) {
  return t < a.total_tiles ? min(t + gstride, a.total_tiles) : a.total_tiles;
}

// The batch kernel's persistent loop for ONE step flavour (Cfg), entered with the first
// tile's header in flight (hc) and, when `synced`, the table in LDS. Software-pipelined
// one tile ahead: while tile i decodes (LDS + VALU only), the header of tile i+2 and the
// code span of tile i+1 are in flight into registers; the span is written to the wave's
// LDS window once tile i has finished reading it. One instantiation per flavour, entered
// with nothing but the first header live (a flavour branch with the first span in
// flight spilled: 80 VGPRs + 40 B of scratch).
template <bool kDelta, class Cfg>
__device__ __forceinline__ void batch_loop(const DecodeArgs &a, uint32_t lane, uint8_t *stage,
                                           const uint8_t *lut, uint32_t t0, uint32_t gstride,
                                           const TileHdr &hc, bool synced MH_TS_PARAM) {
  TileHdr hn;
#if MH_DIAG_STAMPS
  bool first_tile = true;
#endif
  v4u32 R[kStageChunks];
  Tile cur = hdr_resolve(a, hc, lane);
  MH_STAMP(1);
  bool cur_staged = cur.tile < a.total_tiles && cur.span <= (uint32_t)kStageBytes;
  span_issue(a, cur, lane, R, cur_staged);
  hdr_issue(a, next_tile(a, t0, gstride), lane, hn);
  if constexpr (Cfg::kEsc) {  // the general flavour: also an in-kernel table, or a copy loop
    if (!synced) {
      if (a.lut)
        __syncthreads();
      else
        build_lut(a.t1, a.t2, a.t2_entries, s_lut, &s_p0, threadIdx.x, a.nwaves * 64u, [] { __syncthreads(); });
    }
  }
  MH_STAMP(2);
  if (cur_staged) span_write<Cfg::kSwz>(cur, lane, R, stage);
  MH_STAMP(3);
  // Resolved even past the end (zero-record loads): every Tile field is defined
  // before span_issue builds a descriptor from it.
  Tile nxt = hdr_resolve(a, hn, lane);

  // Per iteration the only VMEM issued after a prefetch is the 8 unconditional row
  // stores, so every wait below is an exact vmcnt that leaves the stores in flight.
  while (cur.tile < a.total_tiles) {  // wave-uniform
    if (__builtin_expect(!cur_staged, 0)) break;  // oversize span: finish in the slow loop
    const bool nxt_live = nxt.tile < a.total_tiles;
    const bool nxt_staged = nxt_live && nxt.span <= (uint32_t)kStageBytes;
    span_issue(a, nxt, lane, R, nxt_staged);  // unconditional (all out of range if not staged)
    hdr_issue(a, next_tile(a, nxt.tile, gstride), lane, hn);

    wave_sync();  // this tile's staging writes -> reads
    {
      const bool dead = !cur.valid;
      const OutTile ot = out_tile(a, cur, lane);
      LdsWords src{stage};
      // waves with more tiles left run first (the arbiter otherwise favours the oldest)
      set_prio(min((a.total_tiles - 1u - cur.tile) / gstride, 3u));
      decode_block<kDelta, Cfg>(src, lut, cur.p, cur.init, ot.rsrc, ot.row0, (uint32_t)a.out_pitch, dead);
    }
#if MH_DIAG_STAMPS
    if (first_tile) MH_STAMP(4);
    first_tile = false;
#endif
    wave_sync();  // this tile's reads -> next tile's staging writes
    if (nxt_staged) span_write<Cfg::kSwz>(nxt, lane, R, stage);
    const Tile nn = hdr_resolve(a, hn, lane);
    cur = nxt;
    cur_staged = nxt_staged;
    nxt = nn;
  }

  // Slow loop (rare): a tile whose code span exceeds the LDS window (long codes in
  // most of its 64 blocks) and every later tile of this wave, without prefetch.
  // Kept after the pipelined loop so its waits never merge into that loop.
  for (uint32_t t = cur.tile; t < a.total_tiles; t = next_tile(a, t, gstride)) {
    __builtin_amdgcn_s_waitcnt(0);
    TileHdr h;
    hdr_issue(a, t, lane, h);
    const Tile tt = hdr_resolve(a, h, lane);
    const OutTile ot = out_tile(a, tt, lane);
    decode_halves<kDelta, Cfg>(a, tt, lane, lut, stage, ot.rsrc, ot.row0, !tt.valid);
  }
}

// Flat 8-bit tables (every code 8 bits: all 256 symbols, canonical, so code c is symbol c
// -- the prepared table's flat8 word, which its builder sets only when every first-level
// entry says so, mh_lut.hpp): a block's 64 codes are its 64
// symbol bytes, MSB-first bytes in stream order. A lane decodes its block with byte
// arithmetic -- no table lookup and no serial bit cursor: 17 dwords of codes, realigned
// by v_alignbyte, one SDWA byte add per symbol for the delta sum, 3 VALU per output word.
// The uniform-random 8192^2 stress frame is such a table.
// A tile with a block that does not start on a byte (no reference producer writes one)
// takes a staged funnel-shift step. (Both kernels; the lookup chain for flat tables is the
// round-5 A/B baseline: profiles/r05_flat8_ab.txt, r05_flat8_small_ab.txt.)
struct Flat8Codes {
  uint32_t w[17];  // the block's 64 code bytes from the dword below its first byte
};

__device__ __forceinline__ void flat8_issue(const DecodeArgs &a, const Tile &t, Flat8Codes &c) {
  // unconditional loads (a fixed count, exact vmcnt); a lane without a block reads far
  // past the frame (out of range: 0, no access)
  const __amdgpu_buffer_rsrc_t rc = codes_rsrc(a, t);
  const uint32_t byte = t.start + (t.p >> 3);  // the block's first code byte (frame relative)
  const uint32_t base = t.valid ? (byte & ~3u) : 0xFFFFFF00u;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const v4u32 v = __builtin_amdgcn_raw_buffer_load_b128(rc, (int)(base + 16u * k), 0, 0);
    c.w[4 * k] = v.x;
    c.w[4 * k + 1] = v.y;
    c.w[4 * k + 2] = v.z;
    c.w[4 * k + 3] = v.w;
  }
  c.w[16] = __builtin_amdgcn_raw_buffer_load_b32(rc, (int)(base + 64u), 0, 0);
}

template <bool kDelta>
__device__ __forceinline__ void flat8_block(const DecodeArgs &a, const Tile &t, uint32_t lane, const Flat8Codes &c) {
  typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));
  const uint32_t sb = (t.start + (t.p >> 3)) & 3u;
  const OutTile ot = out_tile(a, t, lane);
  const uint32_t rbase = (t.valid && !MH_DIAG_DROP_STORES) ? ot.row0 : 0x80000000u;
  const uint32_t pitch = (uint32_t)a.out_pitch;
  uint32_t s = t.init;  // running delta sum (byte 0)
#pragma unroll
  for (uint32_t r = 0; r < 8; ++r) {
    // stream bytes 8r .. 8r + 7 (little-endian in each word: byte i = symbol 4j + i)
    const uint32_t c0 = __builtin_amdgcn_alignbyte(c.w[2 * r + 1], c.w[2 * r], sb);
    const uint32_t c1 = __builtin_amdgcn_alignbyte(c.w[2 * r + 2], c.w[2 * r + 1], sb);
    v2u32 v;
    if (kDelta) {
      uint32_t sv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) sv[i] = s = s + ((c0 >> (8 * i)) & 0xFFu);
      v.x = pack_lo4(sv[0], sv[1], sv[2], sv[3]);
#pragma unroll
      for (int i = 0; i < 4; ++i) sv[i] = s = s + ((c1 >> (8 * i)) & 0xFFu);
      v.y = pack_lo4(sv[0], sv[1], sv[2], sv[3]);
    } else {
      v.x = c0;
      v.y = c1;
    }
    __builtin_amdgcn_raw_buffer_store_b64(v, ot.rsrc, (int)(rbase + r * pitch), 0, kBatchStoreAux);
  }
}

// The batch kernel's loop for flat 8-bit tables: the same static tile schedule, software
// pipelined like batch_loop -- while a tile decodes, the next tile's codes and the one
// after's header are in flight, all issued before this tile's row stores, so no wait
// below is for a store.
template <bool kDelta>
__device__ __forceinline__ void flat8_loop(const DecodeArgs &a, uint32_t lane, uint8_t *stage, const uint8_t *lut,
                                           uint32_t t0, uint32_t gstride, const TileHdr &hc MH_TS_PARAM) {
  TileHdr h;
  Flat8Codes cc, cn;
  Tile cur = hdr_resolve(a, hc, lane);
  MH_STAMP(1);
  flat8_issue(a, cur, cc);
  hdr_issue(a, next_tile(a, t0, gstride), lane, h);
#if MH_DIAG_STAMPS
  ts[2] = ts[1];
  ts[3] = ts[1];
  bool first_tile = true;
#endif
  while (cur.tile < a.total_tiles) {  // wave-uniform
    // a block off the byte grid: this tile and the rest in the slow loop below
    if (__builtin_expect(__ballot(cur.valid && ((cur.p & 7u) != 0u)) != 0, 0)) break;
    const Tile nxt = hdr_resolve(a, h, lane);
    flat8_issue(a, nxt, cn);
    hdr_issue(a, next_tile(a, nxt.tile, gstride), lane, h);
    flat8_block<kDelta>(a, cur, lane, cc);
#if MH_DIAG_STAMPS
    if (first_tile) MH_STAMP(4);  // the first tile's codes landed and its stores issued
    first_tile = false;
#endif
    cur = nxt;
    cc = cn;
  }
  // Slow loop (no reference producer gets here): each half tile staged in LDS and decoded
  // with the funnel-shift byte step (any bit alignment), no prefetch; no table needed.
  using Batch8 = StepCfg<kLutBits, true, false, false, kBatchStoreAux, false, true>;
  for (uint32_t t = cur.tile; t < a.total_tiles; t = next_tile(a, t, gstride)) {
    __builtin_amdgcn_s_waitcnt(0);
    TileHdr hs;
    hdr_issue(a, t, lane, hs);
    const Tile tt = hdr_resolve(a, hs, lane);
    const OutTile ot = out_tile(a, tt, lane);
    decode_halves<kDelta, Batch8>(a, tt, lane, lut, stage, ot.rsrc, ot.row0, !tt.valid);
  }
}

// The batch kernel: persistent workgroups (wave w of workgroup g decodes tiles
// g*W + w, + grid*W, ...). A common prologue (table copy, first two headers, first
// span) and then one instantiation of the persistent loop per step flavour, chosen
// from the prepared table's code lengths (kernel-uniform): no code longer than 13 bits
// -> escape-free; one code length only -> escape-free with the swizzled stage. An
// in-kernel table (no prepared LUT) keeps the general step.
template <bool kDelta>
// Leading scalar arguments: preloaded into SGPRs at wave launch (as the small kernel's).
__global__ void __launch_bounds__(64 * kMaxWavesPerWG, kMinWavesPerEU) mh_decode_kernel(
    const uint32_t *p_offsets, const uint64_t *p_frame_off, const uint8_t *p_block_init, const uint16_t *p_lut,
    uint32_t p_nb, uint32_t p_tiles_per_frame, uint32_t p_total_tiles, uint32_t p_nwaves, uint32_t p_grid,
    const DecodeArgs a0) {
  DecodeArgs a = a0;
  a.offsets = p_offsets;
  a.frame_off = p_frame_off;
  a.block_init = p_block_init;
  a.lut = p_lut;
  a.nb = p_nb;
  a.tiles_per_frame = p_tiles_per_frame;
  a.total_tiles = p_total_tiles;
  a.nwaves = p_nwaves;
  a.grid = p_grid;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = a.nwaves;
  const uint32_t nthreads = nwaves * 64u;
  const uint32_t gstride = a.grid * nwaves;
  uint8_t *stage = s_stage + wave * kStageBytes;
  const uint8_t *lut = reinterpret_cast<const uint8_t *>(s_lut);
#if MH_DIAG_STAMPS
  unsigned long long ts[kDiagSlots] = {};
#endif
  MH_STAMP(0);

  const uint32_t t0 = min(blockIdx.x * nwaves + wave, a.total_tiles);
  TileHdr hc;
  // ---- lookup table into LDS (shared by the workgroup) ----
  // A fixed count of unconditional 16-B loads per thread (chunks past the table fall
  // outside the descriptor and return 0), issued FIRST, all in flight together; the
  // first header follows. The table is stored and the workgroup barrier passed as soon
  // as the table's (L2) loads land -- an LDS-only barrier, so no wave waits there for
  // another wave's (HBM, cold) header. Round 3's loop of dependent copies, behind the
  // header, cost 3 L2 round trips plus the slowest header of the workgroup before the
  // first span could be staged (profiles/r04_v3_tile_start_ab.txt). A launch with a
  // prepared table has >= 5 waves per workgroup (smaller ones take the small-launch
  // kernel), so 4 loads per thread cover the table.
  constexpr uint32_t kLutChunks = kLutBytes / 16, kLutPer = 4;
  const bool fixed_copy = a.lut && nthreads * kLutPer >= kLutChunks;
  // The prepared table's [longest, shortest, flat8] word (mh_lut.hpp): the oldest load of
  // the wave (a vector load through the table's descriptor, empty without a prepared table),
  // so it has landed by the time the table's loads have and the decisions below cost the
  // copy no wait. (A scalar load needs a branch or a kernarg pointer to guard the no-table
  // case, and either waits for a scalar round trip before the table's loads go out.)
  const v4u32 lw = __builtin_amdgcn_raw_buffer_load_b128(
      uniform_rsrc(a.lut, a.lut ? (uint32_t)kPreparedBytes : 0u), kMaxLenOff, 0, 0);
  v4u32 L[kLutPer];
  {
    const __amdgpu_buffer_rsrc_t rl = uniform_rsrc(a.lut, fixed_copy ? (uint32_t)kLutBytes : 0u);
#pragma unroll
    for (uint32_t k = 0; k < kLutPer; ++k)
      L[k] = __builtin_amdgcn_raw_buffer_load_b128(rl, (int)((threadIdx.x + k * nthreads) * 16u), 0, 0);
  }
  hdr_issue(a, t0, lane, hc);
  // The step flavour, from the prepared table's code lengths (kernel-uniform):
  //   2: one code length (flat) -> escape-free step, swizzled stage
  //   1: no code over 13 bits   -> escape-free step
  //   0: general step (escapes), also for an in-kernel table
  const uint32_t mx = a.lut ? __builtin_amdgcn_readfirstlane(lw.x) : 16u;
  const uint32_t mn = __builtin_amdgcn_readfirstlane(lw.y), f8 = __builtin_amdgcn_readfirstlane(lw.z);
  // A flat 8-bit identity table (code c = symbol c, the prepared table's flat8 word,
  // mh_lut.hpp) decodes by byte arithmetic with no table in LDS: no copy, no barrier. The
  // table's loads above were issued anyway (before the word is known) and land unused.
  // (The copy stays a block of its own in front of the flavour branch: with the branch
  // first, the compiler hoisted the loops' common header code above it, and the table
  // stores then waited for the header's HBM round trip -- vmcnt(0).)
  // (The stores themselves do not wait for the word: only the barrier does.)
  if (fixed_copy) {
    v4u32 *dstv = reinterpret_cast<v4u32 *>(s_lut);
#pragma unroll
    for (uint32_t k = 0; k < kLutPer; ++k)
      if (threadIdx.x + k * nthreads < kLutChunks) dstv[threadIdx.x + k * nthreads] = L[k];
    if (!f8) lds_barrier();
  } else if (a.lut && !f8) {
    const v4u32 *src = reinterpret_cast<const v4u32 *>(a.lut);
    v4u32 *dstv = reinterpret_cast<v4u32 *>(s_lut);
    for (uint32_t i = threadIdx.x; i < kLutChunks; i += nthreads) dstv[i] = src[i];
  }

  // the escape-free flavours need a prepared table, so a full fixed copy (>= 5 waves)
  const uint32_t flavor = !fixed_copy ? 0u : mx == mn ? 2u : mx <= (uint32_t)kLutBits ? 1u : 0u;
  if (f8)
    flat8_loop<kDelta>(a, lane, stage, lut, t0, gstride, hc MH_TS_ARG);
  else if (flavor == 1)
    batch_loop<kDelta, Lut13NoEsc>(a, lane, stage, lut, t0, gstride, hc, true MH_TS_ARG);
  else if (flavor == 2)
    batch_loop<kDelta, Lut13Flat>(a, lane, stage, lut, t0, gstride, hc, true MH_TS_ARG);
  else
    batch_loop<kDelta, Lut13>(a, lane, stage, lut, t0, gstride, hc, fixed_copy MH_TS_ARG);
#if MH_DIAG_STAMPS
  MH_STAMP(5);
  __builtin_amdgcn_s_waitcnt(0);
  MH_STAMP(6);
  const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID[3:0]
  ts[7] = ((unsigned long long)xcc << 48) | ((unsigned long long)__smid() << 32) | blockIdx.x;
  const uint32_t gw = blockIdx.x * nwaves + wave;
  if (lane == 0 && gw < (uint32_t)kDiagWaves)
    for (int i = 0; i < kDiagSlots; ++i) g_stamps[gw * kDiagSlots + i] = ts[i];
#endif
}

// ---- small launches (<= one wave per SIMD, e.g. one 2048x1536 frame) -------------
// Every wave decodes one tile, one wave per SIMD: the wave's own instruction stream
// (the per-symbol dependency chain and the instructions beside it), not LDS or VALU
// throughput, sets the time. When the table has no code longer than 14 bits the
// single-level 14-bit table drops the escape test. Workgroups of 4 waves (one per
// SIMD; 192 for a 2048x1536 frame) beat 8 (two waves per SIMD, fewer table copies):
// 5.74 vs 5.89 us (profiles/r01_v15_small_step_ab.txt).
constexpr int kSmallWaves = 4;  // waves per workgroup (one tile each)
constexpr int kSmallMaxTilesPerCU = 4;   // launches up to this many tiles per CU
__shared__ __attribute__((aligned(16))) uint16_t s_lut_small[kLut14Entries];  // 14-bit, or 13-bit L1+L2
static_assert(kLutBytes <= kLut14Bytes, "the 13-bit table fits the small kernel's LUT space");

template <bool kDelta>
// The kernel arguments the first loads depend on come first, as scalars: the code object
// preloads the leading kernarg dwords into SGPRs at wave launch (amdgpu-kernarg-preload,
// build.py), so the block-offset and table loads issue without waiting for a scalar load
// of the kernarg segment; the rest of DecodeArgs is read from memory behind them.
__global__ void __launch_bounds__(64 * kSmallWaves) mh_decode_small_kernel(
    const uint32_t *p_offsets, const uint64_t *p_frame_off, const uint8_t *p_block_init, const uint16_t *p_lut,
    uint32_t p_nb, uint32_t p_tiles_per_frame, uint32_t p_total_tiles, const DecodeArgs a0) {
  DecodeArgs a = a0;
  a.offsets = p_offsets;
  a.frame_off = p_frame_off;
  a.block_init = p_block_init;
  a.lut = p_lut;
  a.nb = p_nb;
  a.tiles_per_frame = p_tiles_per_frame;
  a.total_tiles = p_total_tiles;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr uint32_t nwaves = kSmallWaves;  // launched with kSmallWaves waves per workgroup
  uint8_t *stage = s_stage + wave * kStageBytes;
  const uint8_t *lut = reinterpret_cast<const uint8_t *>(s_lut_small);
  const uint8_t *prepared = reinterpret_cast<const uint8_t *>(a.lut);
#if MH_DIAG_STAMPS
  unsigned long long ts[kDiagSlots] = {};
#endif
  MH_STAMP(0);

  // [longest code, shortest code, flat8] (mh_lut.hpp): one scalar load, first used behind
  // the header's loads
  const v4u32 lens = *reinterpret_cast<const v4u32 *>(prepared + kMaxLenOff);
  const uint32_t max_len = lens.x;
  const uint32_t tile = min(blockIdx.x * nwaves + wave, a.total_tiles);
  TileHdr h;
  hdr_issue(a, tile, lane, h);
  const bool l14 = max_len <= (uint32_t)kLut14Bits;
  // Table copy: a fixed count of unconditional 16-B loads per thread (chunks past
  // the table fall outside the descriptor), issued behind the offsets so that the
  // offsets wait below is an exact vmcnt leaving the table loads in flight; the
  // table's L2 round trip overlaps the offsets' HBM one.
  constexpr int kLutLoads = kLut14Bytes / 16 / (64 * kSmallWaves);  // 8
  static_assert(kLut14Bytes == kLutLoads * 16 * 64 * kSmallWaves, "whole table per pass");
  v4u32 L[kLutLoads];
  {
    const __amdgpu_buffer_rsrc_t rl =
        uniform_rsrc(prepared + (l14 ? kLut14Off : 0), l14 ? (uint32_t)kLut14Bytes : (uint32_t)kLutBytes);
#pragma unroll
    for (int k = 0; k < kLutLoads; ++k)
      L[k] = __builtin_amdgcn_raw_buffer_load_b128(rl, (int)((threadIdx.x + 64u * kSmallWaves * k) * 16u), 0, 0);
  }
  const Tile t = hdr_resolve(a, h, lane);
  MH_STAMP(1);
  const bool live = t.tile < a.total_tiles;
  const bool staged = live && t.span <= (uint32_t)kStageBytes;
  v4u32 R[kStageChunks];
  span_issue(a, t, lane, R, staged);
  {
    v4u32 *dst = reinterpret_cast<v4u32 *>(s_lut_small);
#pragma unroll
    for (int k = 0; k < kLutLoads; ++k) dst[threadIdx.x + 64u * kSmallWaves * k] = L[k];
  }
  // table in LDS: an LDS-only barrier (waits lgkmcnt, not vmcnt), so no wave waits here
  // for another wave's span (HBM, cold); each waits for its own span at its first read.
  // (Skipping the copy and barrier for flat tables put a branch on the lengths word in
  // front of the header's loads, which then waited for its scalar round trip: config 2
  // +4 %, the flat single frame gains nothing worth it.)
  lds_barrier();
  MH_STAMP(2);
  // a flat 8-bit identity table (code c = symbol c; the builder sets the word only when
  // every first-level entry says so): byte arithmetic from the staged span (kernel-uniform)
  const bool flat8 = lens.z != 0u;
  if (!live) return;  // no barrier below
  const OutTile ot = out_tile(a, t, lane);
  const __amdgpu_buffer_rsrc_t out = ot.rsrc;
  const uint32_t row0 = ot.row0;
  // the small kernel's step flavours (all with write-through row stores)
  using Small14 = StepCfg<kLut14Bits, false, false, false, kSmallStoreAux, true>;
  using Small13 = StepCfg<kLutBits, false, true, false, kSmallStoreAux, true>;
  using SmallFlat8 = StepCfg<kLutBits, false, false, false, kSmallStoreAux, false, true>;
#if MH_DIAG_STAMPS && MH_DIAG_CLOCK
  unsigned long long c3 = 0;
#endif
  if (staged) {
    span_write(t, lane, R, stage);
    wave_sync();
    MH_STAMP(3);
#if MH_DIAG_STAMPS && MH_DIAG_CLOCK
    c3 = __builtin_amdgcn_s_memtime();
#endif
    LdsWords src{stage};
    if (flat8)
      decode_block<kDelta, SmallFlat8>(src, lut, t.p, t.init, out, row0, (uint32_t)a.out_pitch, !t.valid);
    else if (l14)
      decode_block<kDelta, Small14>(src, lut, t.p, t.init, out, row0, (uint32_t)a.out_pitch, !t.valid);
    else
      decode_block<kDelta, Small13>(src, lut, t.p, t.init, out, row0, (uint32_t)a.out_pitch, !t.valid);
  } else if (flat8) {
    decode_halves<kDelta, SmallFlat8>(a, t, lane, lut, stage, out, row0, !t.valid);
  } else if (l14) {
    decode_halves<kDelta, Small14>(a, t, lane, lut, stage, out, row0, !t.valid);
  } else {
    decode_halves<kDelta, Small13>(a, t, lane, lut, stage, out, row0, !t.valid);
  }
#if MH_DIAG_STAMPS
  MH_STAMP(4);
#if MH_DIAG_CLOCK
  ts[5] = staged ? __builtin_amdgcn_s_memtime() - c3 : 0ull;  // core clocks of the decode
#else
  ts[5] = ts[4];
#endif
  __builtin_amdgcn_s_waitcnt(0);
  MH_STAMP(6);
  const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID[3:0]
  ts[7] = ((unsigned long long)xcc << 48) | ((unsigned long long)__smid() << 32) | blockIdx.x;
  const uint32_t gw = blockIdx.x * nwaves + wave;
  if (lane == 0 && gw < (uint32_t)kDiagWaves)
    for (int i = 0; i < kDiagSlots; ++i) g_stamps[gw * kDiagSlots + i] = ts[i];
#endif
}

#if MH_LANE_PAIRS
// ---- lane-pair variant of the small-launch kernel (MH_FLAG_LANE_PAIRS, A/B) -------
// north_star's lane-group cursor: each 8x8 block is decoded by two lanes of one
// wave, lanes l and l ^ 32 (32 blocks per wave, so twice the waves of the small
// kernel). Lane A starts at the block's first bit (AAPLShaders.metal:241-268);
// lane B starts speculatively at the block's middle bit M = off + len/2 (len from
// the next block's offset). Huffman paths re-synchronise: once A reaches a bit >= M
// at which B also started a symbol, the two paths coincide from there on, so A stops
// and B's symbols from that point are the block's remaining symbols (lp_decode).
// Round 3 rewrite: the round-2 kernel exchanged cursors and
// masks through three ds_bpermutes on every step and stored every symbol to LDS
// (35.7 vs 5.8 us); this one runs the default step with register output and swaps
// the window masks only at sparse checkpoints.
constexpr uint32_t kLpMinBits = 16;  // blocks shorter than 2x this decode on one lane
constexpr int kLpWaves = 4;
constexpr int kLpStageBytes = 4144;   // >= 15 + 32 blocks x 64 x 16 bits / 8 + 24, 16-B multiple
static_assert(kLpStageBytes <= kStageChunks * 64 * 16, "span_issue covers the lane-pair stage");
constexpr int kLpOutStride = 68;      // bytes per lane row (17 dwords: lanes spread over banks)
__shared__ __attribute__((aligned(16))) uint16_t s_lp_lut[kLut14Entries];
__shared__ __attribute__((aligned(16))) uint8_t s_lp_stage[kLpWaves * kLpStageBytes];
__shared__ __attribute__((aligned(16))) uint8_t s_lp_out[kLpWaves * 64 * kLpOutStride];

__device__ __forceinline__ uint32_t lane_xchg(uint32_t lane, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane ^ 32u) << 2), (int)v);
}

// bytewise (mod 256) add of c to the four bytes of b
__device__ __forceinline__ uint32_t add_bytes(uint32_t b, uint32_t c) {
  const uint32_t c4 = c * 0x01010101u;
  return ((b & 0x7F7F7F7Fu) + (c4 & 0x7F7F7F7Fu)) ^ ((b ^ c4) & 0x80808080u);
}

// One block on two lanes (round 3: no per-step exchange).
//   * Both lanes run the default kernel's step (64-bit window, refill before every
//     symbol pair, masked next-word read) in one unrolled 64-step loop, so symbol n
//     goes to a fixed byte of the lane's 16 output registers (v_perm packing).
//   * Each lane records its own symbol starts in the window [mid, mid + 128) as a
//     128-bit mask (a 64-bit window leaves 8.4 % of BigBridge's blocks unmatched, this
//     one 1.4 %; scripts/sim_lane_pairs_ckpt.py). B stops at the block end; A stops at the first start that is also
//     one of B's, which it tests on every step once it holds B's final mask.
//   * B's mask reaches A through five ds_bpermutes at sparse checkpoints (every
//     4 steps from step 8, only while some lane of the wave still waits for it); A
//     lanes that were already past the meeting point by then stop at the checkpoint
//     (first common bit of the two masks; their extra symbols are the block's own).
//   * Afterwards one exchange settles the split: A keeps symbols [0, ia), B supplies
//     [ia, 64) from its own index jb; if B decoded too few (corrupt input, a partner
//     that never synchronised) A finishes the block alone. Rows are assembled from the
//     two lanes' register rows through LDS with dword reads and v_alignbyte; B's
//     running sums are rebased bytewise by the delta sum at the meeting point.
template <bool kDelta, class Cfg>
__device__ __forceinline__ void lp_decode(const uint8_t *stage, const uint8_t *lut, uint32_t *row_a,
                                          uint32_t *row_b, uint32_t lane, bool valid, uint32_t p,
                                          uint32_t mid, uint32_t end, bool spec, uint32_t init,
                                          __amdgpu_buffer_rsrc_t out, uint32_t row0, uint32_t pitch) {
  typedef const __attribute__((address_space(3))) uint8_t *lds_u8;
  typedef const __attribute__((address_space(3))) uint32_t *lds_u32;
  const bool is_b = lane >= 32u;
  const lds_u8 base = (lds_u8)stage;
  const uint32_t s0 = is_b ? mid : p;
  lds_u8 wa = base + (s0 >> 5) * 4u;
  uint32_t wbits = (s0 & ~31u) + Cfg::kCur;  // cursor bit = wbits - (S & 0xFF)
  uint32_t S = ((is_b ? 0u : init) << 8) + Cfg::kCur - (s0 & 31u);
  uint32_t kRefill = Cfg::kRefillAt;
  if constexpr ((Cfg::kRefillAt & 1u) != 0u) asm("s_mov_b32 %0, %1" : "=s"(kRefill) : "n"(Cfg::kRefillAt));
  uint32_t hi = *(lds_u32)wa, lo = *(lds_u32)(wa + 4), nw = *(lds_u32)(wa + 8);
  bool act = valid && (!is_b || spec);
  bool chk = valid && spec && !is_b;  // A: still looking for the meeting point
  bool have = false;                   // A: holds B's final window mask
  uint64_t mine0 = 0, mine1 = 0, other0 = 0, other1 = 0;  // starts at mid + [0,64), [64,128)
  uint32_t nd = 0, srel = 128u;        // symbols decoded; meeting point - mid (128: none)
  uint32_t o[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) o[k] = 0u;

  const auto step = [&](const int n) {
    bool c = false;
    if ((n & 1) == 0) {  // sh < 32 at every pair start (codes <= 16 bits)
      c = (S & 0xFFu) <= kRefill;
      hi = c ? lo : hi;
      lo = c ? nw : lo;
      const uint32_t d = c ? 4u : 0u;
      wa += d;
      wbits += d * 8u;
      S += d * 8u;
    }
    const uint64_t x = (((uint64_t)hi) << 32) | lo;
    uint32_t e = *(const __attribute__((address_space(3))) uint16_t *)(
        (lds_u8)lut + ((uint32_t)(x >> (S & 63u)) & Cfg::kMask));
    if ((n & 1) == 0) nw = *(lds_u32)(wa + 8);
    if constexpr (Cfg::kEsc) {
      const bool esc = e < kEscapeBelow;
      if (__builtin_expect(__ballot(esc) != 0, 0)) {
        const uint32_t x3 = (uint32_t)(x >> ((S - 2u) & 63u)) & 7u;
        const uint32_t e2 = *(const __attribute__((address_space(3))) uint16_t *)(
            (lds_u8)lut + 2u * (kL1Entries + ((e & 0xFFu) << kL2Bits) + x3));
        e = esc ? e2 : e;
      }
    }
    S += e;
    o[n >> 2] = __builtin_amdgcn_perm(kDelta ? S : e + 0xFFu, o[n >> 2], ins_sel1(n & 3));
  };

#pragma unroll
  for (int n = 0; n < 64; ++n) {
    if ((n & 1) == 0 && !__ballot(act)) break;  // wave-uniform
    if (n >= 8 && (n & 3) == 0) {
      const bool need = chk && !have;
      if (__ballot(need)) {
        const uint32_t pos = wbits - (S & 0xFFu);
        const bool fin = !act || (int)(pos - mid) >= 128;  // B: its window mask is final
        const uint32_t xf = lane_xchg(lane, fin ? 1u : 0u);
        const uint32_t x0 = lane_xchg(lane, (uint32_t)mine0);
        const uint32_t x1 = lane_xchg(lane, (uint32_t)(mine0 >> 32));
        const uint32_t x2 = lane_xchg(lane, (uint32_t)mine1);
        const uint32_t x3 = lane_xchg(lane, (uint32_t)(mine1 >> 32));
        if (need && xf) {
          have = true;
          other0 = ((uint64_t)x1 << 32) | x0;
          other1 = ((uint64_t)x3 << 32) | x2;
          const uint64_t c0 = mine0 & other0, c1 = mine1 & other1;
          if (c0 | c1) {  // already past the meeting point
            chk = false;
            act = false;
            srel = c0 ? (uint32_t)__builtin_ctzll(c0) : 64u + (uint32_t)__builtin_ctzll(c1);
          } else if ((int)(pos - mid) >= 128) {
            chk = false;  // passed the window without meeting: A decodes the block alone
          }
        }
      }
    }
    {
      // window bookkeeping, branch-free (selects, no exec-mask branches)
      const uint32_t rel = (wbits - (S & 0xFFu)) - mid;
      const bool inw = act && rel < 128u;
      const uint64_t bit = 1ull << (rel & 63u);
      const uint64_t b0 = (inw && rel < 64u) ? bit : 0ull;
      const uint64_t b1 = (inw && rel >= 64u) ? bit : 0ull;
      const bool look = chk && have;
      const bool hit = look && ((other0 & b0) | (other1 & b1)) != 0ull;
      srel = hit ? rel : srel;
      chk = chk && !hit && !(look && act && !inw && (int)rel >= 128);
      act = act && !hit;
      mine0 |= hit ? 0ull : b0;
      mine1 |= hit ? 0ull : b1;
    }
    if (act) {
      step(n);
      nd = (uint32_t)n + 1u;
      act = !((is_b && (wbits - (S & 0xFFu)) >= end) || n == 63);
    }
  }

  // the split: A's symbols before the meeting point (ia), B's (jb)
  const bool met = !is_b && srel < 128u;
  uint32_t ia = 64u, jb = 0u;
  if (met) {  // A's starts at or after the meeting point; B's before it
    const bool lo = srel < 64u;
    const uint32_t r = srel & 63u;
    ia = nd - (lo ? (uint32_t)__builtin_popcountll(mine0 >> r) + (uint32_t)__builtin_popcountll(mine1)
                  : (uint32_t)__builtin_popcountll(mine1 >> r));
    jb = lo ? (uint32_t)__builtin_popcountll(other0 & ((1ull << r) - 1ull))
            : (uint32_t)__builtin_popcountll(other0) + (uint32_t)__builtin_popcountll(other1 & ((1ull << r) - 1ull));
  }
  const uint32_t nb_b = lane_xchg(lane, nd);
  const bool ok = met && nb_b >= jb + 64u - ia;
  // B decoded too few symbols past the meeting point: A finishes the block alone
  const bool rep = met && !ok;
  if (__ballot(rep)) {
#pragma unroll
    for (int n = 0; n < 64; ++n)
      if (rep && (uint32_t)n >= nd) step(n);
  }
  const uint32_t dec = ok ? (0x80000000u | (ia << 8) | jb) : 0u;
  const uint32_t decx = lane_xchg(lane, dec);
  const uint32_t f = is_b ? decx : dec;
  const bool split = (f >> 31) != 0;
  ia = split ? (f >> 8) & 0x7Fu : 64u;
  jb = f & 0x7Fu;

  uint32_t *row = is_b ? row_b : row_a;
#pragma unroll
  for (int k = 0; k < 16; ++k) row[k] = o[k];
  wave_sync();  // both lanes' rows -> reads
  uint32_t cadd = 0;
  if (kDelta) {
    const uint32_t pa = ia ? reinterpret_cast<const uint8_t *>(row_a)[ia - 1u] : init;
    const uint32_t pb = jb ? reinterpret_cast<const uint8_t *>(row_b)[jb - 1u] : 0u;
    cadd = (pa - pb) & 0xFFu;
  }
  const uint32_t r0 = is_b ? 4u : 0u;
  typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (uint32_t r = 0; r < 4; ++r) {
    v2u32 v;
#pragma unroll
    for (uint32_t h = 0; h < 2; ++h) {
      const uint32_t q = (r0 + r) * 2u + h;
      const uint32_t aw = row_a[q];
      // B byte index of output byte 4q, + 8 (>= 5 whenever a byte of this word is B's;
      // the clamp only keeps all-A words' unused reads inside the LDS rows)
      int u = (int)(4u * q + 8u + jb) - (int)ia;
      u = u < 4 ? 4 : u;
      uint32_t bw = __builtin_amdgcn_alignbyte(row_b[(u >> 2) - 1], row_b[(u >> 2) - 2], (uint32_t)u & 3u);
      if (kDelta) bw = add_bytes(bw, cadd);
      const int na = (int)ia - (int)(4u * q);  // leading bytes of this word from A
      const uint32_t m = na >= 4 ? 0xFFFFFFFFu : na <= 0 ? 0u : (1u << (8 * na)) - 1u;
      const uint32_t w = (aw & m) | (bw & ~m);
      if (h == 0) v.x = w; else v.y = w;
    }
    const uint32_t off = valid ? row0 + (r0 + r) * pitch : 0xFFFFFFF0u;
    __builtin_amdgcn_raw_buffer_store_b64(v, out, (int)off, 0, Cfg::kAux);
  }
}

template <bool kDelta>
__global__ void __launch_bounds__(64 * kLpWaves) mh_decode_lanepair_kernel(const DecodeArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t bl = lane & 31u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t *stage = s_lp_stage + wave * kLpStageBytes;
  uint32_t *row_a = reinterpret_cast<uint32_t *>(s_lp_out + (wave * 64u + bl) * kLpOutStride);
  uint32_t *row_b = reinterpret_cast<uint32_t *>(s_lp_out + (wave * 64u + 32u + bl) * kLpOutStride);
  const uint8_t *lut = reinterpret_cast<const uint8_t *>(s_lp_lut);
  const uint8_t *prepared = reinterpret_cast<const uint8_t *>(a.lut);
  const uint32_t max_len = *reinterpret_cast<const uint32_t *>(prepared + kMaxLenOff);
  const bool l14 = max_len <= (uint32_t)kLut14Bits;

  // header: 32-block tiles (a.tiles_per_frame / a.total_tiles count them)
  const uint32_t tile = __builtin_amdgcn_readfirstlane(min(blockIdx.x * kLpWaves + wave, a.total_tiles));
  const bool live = tile < a.total_tiles;
  const uint32_t fi = live ? tile / a.tiles_per_frame : 0u;
  const uint32_t b0 = live ? (tile - fi * a.tiles_per_frame) * 32u : 0u;
  const uint32_t b = b0 + bl;
  const __amdgpu_buffer_rsrc_t ro = uniform_rsrc(a.offsets + (uint64_t)fi * a.nb, live ? a.nb * 4u : 0u);
  const uint32_t off = __builtin_amdgcn_raw_buffer_load_b32(ro, (int)(b * 4u), 0, 0);
  const uint32_t nxt = __builtin_amdgcn_raw_buffer_load_b32(ro, (int)(b * 4u + 4u), 0, 0);
  typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));
  const __amdgpu_buffer_rsrc_t rf = uniform_rsrc(
      a.frame_off ? (const void *)a.frame_off : (const void *)a.offsets,
      (live && a.frame_off) ? 0x7FFFFFF0u : 0u);
  const v2u32 fo = __builtin_amdgcn_raw_buffer_load_b64(rf, (int)((fi + (lane & 1u)) * 8u), 0, 0);
  const __amdgpu_buffer_rsrc_t ri = uniform_rsrc(
      a.block_init ? (const void *)(a.block_init + (uint64_t)fi * a.nb) : (const void *)a.offsets,
      (live && a.block_init) ? a.nb : 0u);
  const uint32_t init = __builtin_amdgcn_raw_buffer_load_b8(ri, (int)b, 0, 0) & 0xFFu;
  // table copy, unconditional 16-B loads issued behind the header (as the small kernel)
  constexpr int kLutLoads = kLut14Bytes / 16 / (64 * kLpWaves);
  static_assert(kLut14Bytes == kLutLoads * 16 * 64 * kLpWaves, "whole table per pass");
  v4u32 L[kLutLoads];
  {
    const __amdgpu_buffer_rsrc_t rl =
        uniform_rsrc(prepared + (l14 ? kLut14Off : 0), l14 ? (uint32_t)kLut14Bytes : (uint32_t)kLutBytes);
#pragma unroll
    for (int k = 0; k < kLutLoads; ++k)
      L[k] = __builtin_amdgcn_raw_buffer_load_b128(rl, (int)((threadIdx.x + 64u * kLpWaves * k) * 16u), 0, 0);
  }
  Tile t;
  t.tile = tile;
  t.f = fi;
  t.b0 = b0;
  t.valid = live && b < a.nb;
  uint64_t fbytes = a.codes_bytes;
  t.fbeg = 0;
  if (a.frame_off) {
    const uint64_t lo = ((uint64_t)__builtin_amdgcn_readlane(fo.y, 0) << 32) | __builtin_amdgcn_readlane(fo.x, 0);
    const uint64_t hi = ((uint64_t)__builtin_amdgcn_readlane(fo.y, 1) << 32) | __builtin_amdgcn_readlane(fo.x, 1);
    t.fbeg = lo;
    fbytes = hi - lo;
  }
  t.fb32 = (uint32_t)(fbytes > 0xFFFFFFF0ull ? 0xFFFFFFF0ull : fbytes);
  const uint32_t fbits = t.fb32 > 0x1FFFFFFFu ? 0xFFFFFFFFu : t.fb32 * 8u;
  const bool exact_end = b + 1u < a.nb;
  const uint32_t end_l = exact_end ? nxt : min(fbits, off + 64u * 16u);
  const uint32_t last = live ? min(31u, a.nb - 1u - b0) : 0u;
  const uint32_t sb = __builtin_amdgcn_readfirstlane(off);
  const uint32_t eb = __builtin_amdgcn_readlane(end_l, last);
  t.start = (sb >> 3) & ~15u;
  uint32_t endb = (eb >> 3) + 24u;
  if (endb > t.fb32 + 16u) endb = t.fb32 + 16u;
  t.span = endb > t.start ? min((endb - t.start + 15u) & ~15u, (uint32_t)kLpStageBytes) : 0u;
  t.p = t.valid ? off - t.start * 8u : 0u;
  t.init = init;
  v4u32 R[kStageChunks];
  span_issue(a, t, lane, R, live);
  {
    v4u32 *dst = reinterpret_cast<v4u32 *>(s_lp_lut);
#pragma unroll
    for (int k = 0; k < kLutLoads; ++k) dst[threadIdx.x + 64u * kLpWaves * k] = L[k];
  }
  __syncthreads();  // table in LDS
  if (!live) return;  // wave-uniform; no barrier below
  span_write(t, lane, R, stage);
  wave_sync();
  // output: descriptor at the tile's first block row (as out_tile, 32-block tiles)
  const uint32_t bx = b % a.bw, by = b / a.bw;
  const uint32_t by0 = __builtin_amdgcn_readfirstlane(b0 / a.bw);
  const uint64_t base = (uint64_t)by0 * 8u * a.out_pitch;
  const uint64_t rem = a.out_frame_bytes > base ? a.out_frame_bytes - base : 0u;
  const __amdgpu_buffer_rsrc_t out = uniform_rsrc(a.out + (uint64_t)fi * a.out_frame_stride + base,
                                                  (uint32_t)(rem < 0x7FFFFFF0ull ? rem : 0x7FFFFFF0ull));
  const uint32_t row0 = (by - by0) * 8u * (uint32_t)a.out_pitch + bx * 8u;
  const uint32_t len = end_l - off;
  const uint32_t mid = t.p + (len >> 1);
  const uint32_t end = t.p + len;
  // the frame's last block has no exact end: lane A alone
  const bool spec = t.valid && exact_end && len >= 2u * kLpMinBits && len <= 64u * 16u;
  if (l14)
    lp_decode<kDelta, StepCfg<kLut14Bits, false, false>>(stage, lut, row_a, row_b, lane, t.valid, t.p, mid, end,
                                                  spec, init, out, row0, (uint32_t)a.out_pitch);
  else
    lp_decode<kDelta, StepCfg<kLutBits, false, true>>(stage, lut, row_a, row_b, lane, t.valid, t.p, mid, end,
                                                spec, init, out, row0, (uint32_t)a.out_pitch);
}

#endif  // MH_LANE_PAIRS

// Per-device launch parameters (CU count, batch-kernel occupancy per workgroup
// size), computed once per device ordinal under a per-device mutex: no mutable state
// is shared between devices or written by concurrent callers (the reference keeps
// its tables in module statics, Shared/HuffmanUtil.cpp:87-102).
constexpr int kMaxDevices = 64;
struct DeviceInfo {
  std::mutex m;
  std::atomic<int> cus{0};  // nonzero once the entry is complete
  int occ[2][kMaxWavesPerWG + 1] = {};
};
DeviceInfo g_devinfo[kMaxDevices];

template <bool kDelta>
int occupancy_query(int nw) {
  int blocks = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, mh_decode_kernel<kDelta>, nw * 64, 0) !=
          hipSuccess ||
      blocks < 1)
    blocks = 1;
  return blocks;
}

// The device a launch on `s` runs on (the stream's, or the caller's current one).
int stream_device(hipStream_t s) {
  int dev = -1;
  if (s && hipStreamGetDevice(s, &dev) == hipSuccess) return dev;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  return dev;
}

// Filled once per device under its mutex; a failed query leaves the entry empty,
// so the next call tries again (a transient HIP error does not stick).
const DeviceInfo *device_info(hipStream_t s) {
  const int dev = stream_device(s);
  if (dev < 0 || dev >= kMaxDevices) return nullptr;
  DeviceInfo &d = g_devinfo[dev];
  if (d.cus.load(std::memory_order_acquire)) return &d;
  std::lock_guard<std::mutex> lock(d.m);
  if (d.cus.load(std::memory_order_relaxed)) return &d;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess || prop.multiProcessorCount < 1) return nullptr;
  int cur = -1;
  const bool swap = hipGetDevice(&cur) == hipSuccess && cur != dev;
  if (swap && hipSetDevice(dev) != hipSuccess) return nullptr;
  for (int nw = 1; nw <= kMaxWavesPerWG; ++nw) {
    d.occ[0][nw] = occupancy_query<false>(nw);
    d.occ[1][nw] = occupancy_query<true>(nw);
  }
  if (swap) (void)hipSetDevice(cur);
  d.cus.store(prop.multiProcessorCount, std::memory_order_release);  // last: marks the entry complete
  return &d;
}

// One kernel launch; any_order (MH_FLAG_ANY_ORDER) clears the dispatch packet's
// barrier bit so the kernel may start while earlier work on the stream drains.
#define MH_LAUNCH(kernel, grid, block, s, any_order, ...)                                          \
  do {                                                                                            \
    if (any_order)                                                                                \
      hipExtLaunchKernelGGL(kernel, grid, block, 0, s, nullptr, nullptr, hipExtAnyOrderLaunch, __VA_ARGS__); \
    else                                                                                          \
      hipLaunchKernelGGL(kernel, grid, block, 0, s, __VA_ARGS__);                                 \
  } while (0)

template <bool kDelta>
int launch(const DecodeArgs &a0, hipStream_t s, bool lane_pairs, bool any_order) {
  DecodeArgs a = a0;
  const DeviceInfo *di = device_info(s);
  if (!di) return MH_ERR_HIP;
  const int cus = di->cus.load(std::memory_order_relaxed);
#if MH_LANE_PAIRS
  if (lane_pairs && a.lut && a.total_tiles <= (uint32_t)(kSmallMaxTilesPerCU * cus)) {
    // experimental lane-pair decode (MH_FLAG_LANE_PAIRS): 32-block tiles
    const uint32_t n_frames = a.total_tiles / a.tiles_per_frame;
    a.tiles_per_frame = (a.nb + 31u) / 32u;
    a.total_tiles = a.tiles_per_frame * n_frames;
    a.n_groups = (a.total_tiles + kLpWaves - 1) / kLpWaves;
    MH_LAUNCH(mh_decode_lanepair_kernel<kDelta>, dim3(a.n_groups), dim3(kLpWaves * 64), s, any_order, a);
    return hipGetLastError() == hipSuccess ? MH_OK : MH_ERR_HIP;
  }
#else
  (void)lane_pairs;
#endif
  if (a.lut && a.total_tiles <= (uint32_t)(kSmallMaxTilesPerCU * cus)) {
    // one tile per wave, kSmallWaves waves per workgroup: fewer workgroups copy the
    // table (measured: 8-wave groups beat one 3-wave group per CU by ~5 %)
    const uint32_t nw = kSmallWaves;
    a.n_groups = (a.total_tiles + nw - 1) / nw;
    MH_LAUNCH(mh_decode_small_kernel<kDelta>, dim3(a.n_groups), dim3(nw * 64), s, any_order, a.offsets,
              a.frame_off, a.block_init, a.lut, a.nb, a.tiles_per_frame, a.total_tiles, a);
    return hipGetLastError() == hipSuccess ? MH_OK : MH_ERR_HIP;
  }
  // Waves per workgroup: spread a small launch (one 2048x1536 frame = 768 tiles)
  // over every CU; 8-wave workgroups (3 per CU by LDS) for batches.
  uint32_t nw = (a.total_tiles + (uint32_t)cus - 1) / (uint32_t)cus;
  if (nw < 1) nw = 1;
  if (nw > (uint32_t)kMaxWavesPerWG) nw = kMaxWavesPerWG;
  a.n_groups = (a.total_tiles + nw - 1) / nw;
  const uint32_t resident = (uint32_t)(cus * di->occ[kDelta ? 1 : 0][nw]);
  const uint32_t grid = a.n_groups < resident ? a.n_groups : resident;
  a.nwaves = nw;
  a.grid = grid;
  MH_LAUNCH(mh_decode_kernel<kDelta>, dim3(grid), dim3(nw * 64), s, any_order, a.offsets, a.frame_off,
            a.block_init, a.lut, a.nb, a.tiles_per_frame, a.total_tiles, a.nwaves, a.grid, a);
  return hipGetLastError() == hipSuccess ? MH_OK : MH_ERR_HIP;
}

}  // namespace

extern "C" {

#if !MH_LANE_PAIRS

#if MH_DIAG_STAMPS
int mh_diag_stamps(unsigned long long *host, size_t n) {
  if (n > sizeof(g_stamps) / sizeof(g_stamps[0])) n = sizeof(g_stamps) / sizeof(g_stamps[0]);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), n * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? (int)n : -1;
}
#endif

#ifdef MH_TABLE_STAMPS  // diagnostic builds: room for the table kernel's phase stamps
size_t mh_lut_bytes(void) { return (size_t)kPreparedBytes + 256; }
#else
size_t mh_lut_bytes(void) { return (size_t)kPreparedBytes; }
#endif
int mh_lut_bits(void) { return kLutBits; }

int mh_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int mh_prepare_lut(const mh_lookup_symbol *d_table1, const mh_lookup_symbol *d_table2,
                   uint32_t table2_entries, uint16_t *d_lut, void *stream) {
  if (!d_table1 || !d_table2 || !d_lut) return MH_ERR_INVALID_ARG;
  if (table2_entries < 256 || (table2_entries % 256) != 0 || table2_entries > MH_TABLE2_MAX_ENTRIES)
    return MH_ERR_TABLE;
  if ((uintptr_t)d_lut & 15u) return MH_ERR_ALIGN;
  hipLaunchKernelGGL(mh_prepare_lut_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream,
                     reinterpret_cast<const uint16_t *>(d_table1),
                     reinterpret_cast<const uint16_t *>(d_table2), table2_entries,
                     reinterpret_cast<uint8_t *>(d_lut));
  return hipGetLastError() == hipSuccess ? MH_OK : MH_ERR_HIP;
}

#endif  // !MH_LANE_PAIRS

// The decode entry point. The lane-pair diagnostic library exports the same body as
// mh_diag_decode_lanepairs (and nothing else): MH_FLAG_LANE_PAIRS is honoured only there;
// mh_decode accepts and ignores it.
#if MH_LANE_PAIRS
int mh_diag_decode_lanepairs(const mh_frame *fr, uint8_t *d_out, size_t out_pitch, size_t out_frame_stride,
                             void *stream) {
#else
int mh_decode(const mh_frame *fr, uint8_t *d_out, size_t out_pitch, size_t out_frame_stride,
              void *stream) {
#endif
  if (!fr || !d_out || !fr->d_block_offsets || !fr->d_codes || !fr->d_table1 || !fr->d_table2)
    return MH_ERR_INVALID_ARG;
  if (fr->n_frames == 0 || (fr->n_frames > 1 && !fr->d_frame_code_offsets)) return MH_ERR_INVALID_ARG;
  // MH_FLAG_LANE_PAIRS: honoured by the diagnostic library only; the product library accepts
  // it (callers built against round-4 libraries pass it) and decodes with the default kernels
  if (fr->flags & ~(MH_FLAG_NO_DELTA | MH_FLAG_ANY_ORDER | MH_FLAG_LANE_PAIRS)) return MH_ERR_INVALID_ARG;
  const mh_dims &d = fr->dims;
  if (!d.width || !d.height || d.width > MH_MAX_DIM || d.height > MH_MAX_DIM ||
      d.block_width != (d.width + 7) / 8 || d.block_height != (d.height + 7) / 8)
    return MH_ERR_DIMS;
  if (fr->table2_entries < 256 || (fr->table2_entries % 256) != 0 ||
      fr->table2_entries > MH_TABLE2_MAX_ENTRIES)
    return MH_ERR_TABLE;
  if (((uintptr_t)fr->d_codes & 15u) || (out_pitch & 7u) || ((uintptr_t)d_out & 7u) ||
      (fr->n_frames > 1 && (out_frame_stride & 7u)) || ((uintptr_t)fr->d_lut & 15u))
    return MH_ERR_ALIGN;
  if (out_pitch < d.width || out_pitch > (1u << 20) ||
      (fr->n_frames > 1 && out_frame_stride < out_pitch * d.height))
    return MH_ERR_CAPACITY;
  if (fr->codes_bytes < MH_CODES_PAD) return MH_ERR_CAPACITY;
  if (fr->n_frames == 1 && !fr->d_frame_code_offsets && fr->codes_bytes > 0xFFFFFFF0ull)
    return MH_ERR_CAPACITY;

  DecodeArgs a{};
  a.offsets = fr->d_block_offsets;
  a.codes = fr->d_codes;
  a.frame_off = fr->d_frame_code_offsets;
  a.codes_bytes = fr->codes_bytes;
  a.t1 = reinterpret_cast<const uint16_t *>(fr->d_table1);
  a.t2 = reinterpret_cast<const uint16_t *>(fr->d_table2);
  a.lut = fr->d_lut;
  a.block_init = fr->d_block_init;
  a.out = d_out;
  a.out_pitch = out_pitch;
  a.out_frame_stride = out_frame_stride;
  a.out_frame_bytes = (uint64_t)d.height * out_pitch;
  a.t2_entries = fr->table2_entries;
  a.w = d.width;
  a.h = d.height;
  a.bw = d.block_width;
  a.bh = d.block_height;
  a.nb = d.block_width * d.block_height;
  a.tiles_per_frame = (a.nb + 63) / 64;
  const uint64_t total = (uint64_t)a.tiles_per_frame * fr->n_frames;
  if (total > 0x7FFFFFFFull) return MH_ERR_CAPACITY;
  a.total_tiles = (uint32_t)total;
  hipStream_t s = (hipStream_t)stream;
  const bool lp = (fr->flags & MH_FLAG_LANE_PAIRS) != 0;
  const bool ao = (fr->flags & MH_FLAG_ANY_ORDER) != 0;
  return (fr->flags & MH_FLAG_NO_DELTA) ? launch<false>(a, s, lp, ao) : launch<true>(a, s, lp, ao);
}

}  // extern "C"

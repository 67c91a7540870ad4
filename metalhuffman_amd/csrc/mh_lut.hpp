// mh_lut.hpp -- the decoder's prepared table (mh_prepare_lut's buffer): layout,
// entry format and its construction from T1/T2. Shared by mh_decode.hip (the
// mh_prepare_lut kernel over T1/T2 in device memory) and mh_tables.hip (built
// straight from the tables it just made in LDS).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kLutBits = 13;                  // first-level index width
constexpr int kL1Entries = 1 << kLutBits;     // 8192 x u16
constexpr int kL2Bits = 16 - kLutBits;        // 3 more window bits for long codes
constexpr int kL2Subtables = 129;             // dummy + <=128 long-code prefixes
constexpr int kL2Entries = kL2Subtables << kL2Bits;      // 1032
constexpr int kLutEntries = kL1Entries + 1040;           // L1 + L2, padded to 16 B
constexpr int kLutBytes = kLutEntries * 2;               // 18464: the 13-bit table
// The prepared table buffer (mh_prepare_lut) also holds a single-level 14-bit
// table (no escapes; valid when no code exceeds 14 bits) and the longest code
// length, for the small-launch kernel.
constexpr int kLut14Bits = 14;
constexpr int kLut14Entries = 1 << kLut14Bits;           // 16384 x u16
constexpr int kLut14Off = kLutBytes;                     // byte offset in the buffer
constexpr int kLut14Bytes = kLut14Entries * 2;           // 32768
constexpr int kMaxLenOff = kLut14Off + kLut14Bytes;      // u32 longest, shortest code length, flat-8 flag
constexpr int kPreparedBytes = kMaxLenOff + 16;          // 51248
static_assert(kLutBytes % 16 == 0 && kLut14Bytes % 16 == 0, "lut copy uses 16-byte chunks");
static_assert(kL2Subtables < 240, "escape entries must stay below the smallest step word");

// LUT entry format ("step word"): a valid {symbol, bitWidth} becomes
//   E = (symbol << 8) - bitWidth  (mod 2^16),
// so ONE add of E to the lane state S (see decode_block) advances the bit cursor
// (low byte) and folds the delta into prev (byte 1). Valid entries have a low
// byte in [240, 255] (bitWidth 1..16), so E >= 240. Escapes to the second level
// are E = sub < 129, and a window the table does not decode ({0,0} in the
// reference) is E = 0: adding it changes nothing, exactly the reference's
// zero-width step.
__device__ __forceinline__ uint32_t step_word(uint32_t e) {
  const uint32_t len = e >> 8;
  return len ? (((e & 0xFFu) << 8) - len) & 0xFFFFu : 0u;
}
constexpr uint32_t kEscapeBelow = 240u;

// split_lookup for kBatch windows at once, T1 from LDS: every T2 read is issued
// before any is used (one L2 round trip per batch instead of one per window).
template <int kBatch>
__device__ __forceinline__ void split_lookup_batch(const uint16_t *s_t1, const uint16_t *t2,
                                                   uint32_t t2_entries, const uint32_t (&pat16)[kBatch],
                                                   uint32_t (&e)[kBatch]) {
  uint32_t idx[kBatch];
#pragma unroll
  for (int k = 0; k < kBatch; ++k) {
    e[k] = s_t1[pat16[k] >> 8];
    idx[k] = (e[k] & 0xFFu) * 256u + (pat16[k] & 0xFFu);
  }
  uint32_t v[kBatch];
#pragma unroll
  for (int k = 0; k < kBatch; ++k) v[k] = t2[idx[k] < t2_entries ? idx[k] : 0u];
#pragma unroll
  for (int k = 0; k < kBatch; ++k)
    if ((e[k] >> 8) == 0) e[k] = idx[k] < t2_entries ? v[k] : 0u;
}

// The prepared buffer from T1 (in LDS) and T2 (LDS or global, t2_entries long;
// reads past it are the all-zero entry), by the whole workgroup:
//   L1[p] (p = 13-bit prefix): step_word of the window p << 3 when its code has
//     <= 13 bits or the window is invalid (0 = no-op, as the reference's dummy T2
//     subtable, HuffmanUtil.cpp:550-556); from the first prefix P0 of a longer code
//     on, an escape `sub` into L2[sub*8 + x] (the <= 128 long-code prefixes);
//   the single-level 14-bit table (0 for codes over 14 bits);
//   [longest code, shortest code, flat8, 0] at kMaxLenOff, flat8 = 1 when every first-level
//     entry is the identity 8-bit code (prefix p decodes symbol p >> 5 in 8 bits: all 256
//     symbols, code c = symbol c), the byte-arithmetic decode's condition. The decoder reads
//     this word instead of re-checking the table at every launch.
// Lookups go in batches of 8 with every T2 read issued before any is used.
// `scratch`: 4 words of LDS.
__device__ __forceinline__ void build_prepared_lut(const uint16_t *s_t1, const uint16_t *t2, uint32_t t2_entries,
                                                   uint8_t *buf, uint32_t *scratch) {
  constexpr int kB = 8;
  uint32_t &p0 = scratch[0], &mx = scratch[1], &mn = scratch[2], &flat = scratch[3];
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
  uint16_t *lut = reinterpret_cast<uint16_t *>(buf);
  uint16_t *lut14 = reinterpret_cast<uint16_t *>(buf + kLut14Off);
  if (tid == 0) {
    p0 = (uint32_t)kL1Entries;
    mx = 0;
    mn = 255;
    flat = 1;
  }
  __syncthreads();
  // first level of the 13-bit table and the 14-bit table
  uint32_t my_p0 = (uint32_t)kL1Entries, my_mx = 0, my_mn = 255, my_flat = 1;
  for (uint32_t base = tid * kB; base < (uint32_t)kL1Entries; base += nt * kB) {
    uint32_t pat[kB], e[kB];
#pragma unroll
    for (int k = 0; k < kB; ++k) pat[k] = (base + k) << kL2Bits;
    split_lookup_batch(s_t1, t2, t2_entries, pat, e);
#pragma unroll
    for (int k = 0; k < kB; ++k) {
      const uint32_t sw = step_word(e[k]);
      lut[base + k] = (uint16_t)sw;
      if ((e[k] >> 8) > (uint32_t)kLutBits) my_p0 = min(my_p0, base + k);
      my_flat &= (uint32_t)(sw == (((((base + k) >> (kLutBits - 8)) << 8) - 8u) & 0xFFFFu));
    }
  }
  for (uint32_t base = tid * kB; base < (uint32_t)kLut14Entries; base += nt * kB) {
    uint32_t pat[kB], e[kB];
#pragma unroll
    for (int k = 0; k < kB; ++k) pat[k] = (base + k) << (16 - kLut14Bits);
    split_lookup_batch(s_t1, t2, t2_entries, pat, e);
#pragma unroll
    for (int k = 0; k < kB; ++k) {
      const uint32_t len = e[k] >> 8;
      lut14[base + k] = (uint16_t)(len <= (uint32_t)kLut14Bits ? step_word(e[k]) : 0u);
      my_mx = max(my_mx, len);
      if (len) my_mn = min(my_mn, len);
    }
  }
  for (uint32_t i = tid; i < (uint32_t)(kLutEntries - kL1Entries); i += nt) lut[kL1Entries + i] = 0;
  // wave reductions first: a thousand LDS atomics on one word serialise
  for (uint32_t o = 32; o; o >>= 1) {
    my_p0 = min(my_p0, (uint32_t)__shfl_xor(my_p0, o));
    my_mx = max(my_mx, (uint32_t)__shfl_xor(my_mx, o));
    my_mn = min(my_mn, (uint32_t)__shfl_xor(my_mn, o));
    my_flat &= (uint32_t)__shfl_xor(my_flat, o);
  }
  if ((tid & 63u) == 0) {
    atomicMin(&p0, my_p0);
    atomicMax(&mx, my_mx);
    atomicMin(&mn, my_mn);
    if (!my_flat) flat = 0;
  }
  __syncthreads();
  // escapes and the second level (the long codes), as build_lut
  const uint32_t P0 = p0;
  for (uint32_t p = P0 + tid; p < (uint32_t)kL1Entries; p += nt) {
    const uint32_t sub = p - P0 + 1;
    lut[p] = (uint16_t)(sub < (uint32_t)kL2Subtables ? sub : 0u);
  }
  const uint32_t nl2 = ((uint32_t)kL1Entries - P0) << kL2Bits;
  for (uint32_t i = tid; i < nl2 && i < (uint32_t)(kL2Entries - (1 << kL2Bits)); i += nt) {
    uint32_t pat[1] = {(P0 << kL2Bits) + i}, e[1];
    split_lookup_batch(s_t1, t2, t2_entries, pat, e);
    lut[kL1Entries + (1 << kL2Bits) + i] = (uint16_t)step_word(e[0]);
  }
  // [longest code, shortest code, flat8, 0]
  if (tid < 4)
    reinterpret_cast<uint32_t *>(buf + kMaxLenOff)[tid] = tid == 0 ? mx : tid == 1 ? mn : tid == 2 ? flat : 0u;
}

}  // namespace

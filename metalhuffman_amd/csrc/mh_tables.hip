// mh_tables.hip -- GPU-side table build from the 256-byte canonical header
// (SURVEY.md 8(f) rank 1): each GPU rebuilds T1/T2 and the decoder's prepared
// table from the header, so a multi-GPU job broadcasts 256 bytes instead of T1||T2.
//
// Semantics follow the host builder (mh_host.cpp: mh_build_tables), itself the
// restatement of the reference's canonical-code and split-table construction:
//   canonical codes  huff_util.hpp:94-193 / HuffmanUtil.cpp:270-310 -- symbols sorted
//                    by (length, symbol); the code increments per symbol and shifts
//                    left on every length increase; left-justified to 16 bits;
//   T1 / T2          HuffmanUtil.cpp:338-667 -- T1[hi byte] = {symbol, len} for codes
//                    of <= 8 bits; long codes are grouped by their high byte, groups
//                    numbered 1.. in ascending high-byte order, T1[hi] = {group, 0},
//                    T2[group*256 + lo] = {symbol, len}; T2 subtable 0 is all zero.
// For a header whose code lengths form a prefix code (every encoder output), each
// table slot is written by at most one symbol, so one thread per symbol fills its
// range without ordering concerns. Everything is built in LDS (T2's whole capacity,
// 131.5 KB, fits gfx950's LDS) and written out once. Headers that are not prefix codes (Kraft sum
// > 1) or hold a length > 16 are rejected with a status word.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "../../include/metalhuffman.h"
#include "mh_lut.hpp"

namespace {

// Every workgroup builds T1 and the used part of T2 in LDS; workgroup 0 writes them
// out with 16-byte stores (T2 zero-padded to its whole capacity), and -- when `lut` is given -- each workgroup then
// fills its slice of the decoder's prepared table straight from its LDS copies
// (the same entries as mh_prepare_lut over the written tables, tests/test_gpu_tables.py):
// the prepared table's ~25 K entries are spread over the grid instead of one CU.
// P0 (the first 13-bit prefix of a code longer than 13 bits) and the longest /
// shortest code words come from the canonical codes themselves, so the slices need
// no exchange. Launch: kTableGroups workgroups of 1024 threads.
constexpr uint32_t kTableGroups = 32;
__global__ void __launch_bounds__(1024) mh_build_tables_kernel(const uint8_t *canon, uint16_t *t1,
                                                               uint16_t *t2, uint32_t *t2_entries,
                                                               int32_t *status, uint8_t *lut) {
  __shared__ __attribute__((aligned(16))) uint16_t s_t2[MH_TABLE2_MAX_ENTRIES];
  __shared__ __attribute__((aligned(16))) uint16_t s_t1[256];
  __shared__ uint32_t s_group[256], s_wcnt[4][17], s_gcnt[4];
  __shared__ uint32_t s_first[17], s_bad, s_ngroups, s_mx, s_mn;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
#ifdef MH_TABLE_STAMPS
#define TAB_STAMP(i) \
  if (lut && blockIdx.x == 0 && tid == 0) reinterpret_cast<uint64_t *>(lut + kPreparedBytes)[i] = __builtin_amdgcn_s_memtime();
  TAB_STAMP(0);
#else
#define TAB_STAMP(i)
#endif
  const uint64_t below = (1ull << lane) - 1ull;
  static_assert(MH_TABLE2_MAX_ENTRIES % 8 == 0, "16-byte copies");
  constexpr uint32_t kT2Vec = MH_TABLE2_MAX_ENTRIES / 8;

  uint4 *s_t2v = reinterpret_cast<uint4 *>(s_t2);
  const uint32_t L = tid < 256 ? canon[tid] : 0u;
  if (tid < 256) {
    s_t1[tid] = 0;
    s_group[tid] = 0;
  }
  if (tid == 0) {
    s_bad = 0;
    s_mx = 0;
    s_mn = 255;
  }
  __syncthreads();
  TAB_STAMP(1);
  // codes per length and each symbol's rank among equal lengths (symbol order):
  // one ballot per length per wave
  uint32_t in_wave = 0;
  if (tid < 256) {
    // (no LDS atomics on one word here: 256 of them serialise, ~18 clocks each)
    if (__ballot(L > 16) && lane == 0) s_bad = 1u;
    for (uint32_t l = 1; l <= 16; ++l) {
      const uint64_t m = __ballot(L == l);
      if (L == l) in_wave = (uint32_t)__popcll(m & below);
      if (lane == 0) s_wcnt[wave][l] = (uint32_t)__popcll(m);
    }
  }
  __syncthreads();
  TAB_STAMP(2);
  if (tid < 64) {
    // first code of each length, the recurrence code = (code + count) << 1 in closed
    // form: first[l] = sum over j < l of count[j] << (l - j), a 16-lane prefix sum of
    // count[j] << (16 - j) (<= 2^23) shifted back down
    const uint32_t ln = (tid & 15u) + 1u;
    const uint32_t cnt = tid < 16 ? s_wcnt[0][ln] + s_wcnt[1][ln] + s_wcnt[2][ln] + s_wcnt[3][ln] : 0u;
    const uint32_t v = cnt << (16 - ln);
    uint32_t incl = v;
#pragma unroll
    for (uint32_t d = 1; d < 16; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d);
      if ((tid & 63u) >= d) incl += y;
    }
    if (tid < 16) s_first[ln] = (incl - v) >> (16 - ln);
    if (tid == 15 && incl > 65536u) s_bad |= 2u;  // Kraft sum over 1: not a prefix code
  }
  __syncthreads();
  TAB_STAMP(3);
  const bool bad = s_bad != 0;  // rejected: the tables stay all zero
  uint32_t code = 0;
  if (!bad && tid < 256 && L) {
    uint32_t rank = in_wave;  // symbols of the same length before this one
    for (uint32_t w = 0; w < wave; ++w) rank += s_wcnt[w][L];
    code = ((s_first[L] + rank) << (16 - L)) & 0xFFFFu;
  }
  {
    // longest / shortest code as mh_prepare_lut samples them (windows at multiples
    // of 4): a code of <= 14 bits always holds one, a 15/16-bit code iff it starts
    // there. Wave reductions first: 256 LDS atomics on one word serialise.
    const bool seen = !bad && tid < 256 && L && (L <= 14 || (code & 3u) == 0);
    uint32_t vmx = seen ? L : 0u, vmn = seen ? L : 255u;
    for (uint32_t o = 32; o; o >>= 1) {
      vmx = max(vmx, (uint32_t)__shfl_xor(vmx, o));
      vmn = min(vmn, (uint32_t)__shfl_xor(vmn, o));
    }
    if (tid < 256 && lane == 0) {
      atomicMax(&s_mx, vmx);
      atomicMin(&s_mn, vmn);
    }
  }
  // long codes grouped by high byte, groups numbered 1.. in ascending high-byte order
  if (!bad && tid < 256 && L > 8) s_group[code >> 8] = 1;  // (every writer of a slot stores 1)
  __syncthreads();
  TAB_STAMP(4);
  uint32_t mark = 0, gpre = 0;
  if (tid < 256) {
    mark = s_group[tid];
    const uint64_t m = __ballot(mark != 0);
    gpre = (uint32_t)__popcll(m & below);
    if (lane == 0) s_gcnt[wave] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  TAB_STAMP(5);
  if (tid < 256) {
    uint32_t g = gpre;
    for (uint32_t w = 0; w < wave; ++w) g += s_gcnt[w];
    s_group[tid] = mark ? g + 1u : 0u;
    if (tid == 255) s_ngroups = g + mark;
  }
  __syncthreads();
  TAB_STAMP(6);
  // only the used subtables (dummy + one per group) are ever read: zero just those
  const uint32_t used_vec = (s_ngroups + 1u) * 32u;
  for (uint32_t i = tid; i < used_vec; i += blockDim.x) s_t2v[i] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  TAB_STAMP(7);
  if (!bad && tid < 256 && L) {
    // a code's range is aligned to its size: ranges of >= 8 entries go out as
    // 16-byte LDS stores (a 9-bit code: 16 stores, not 128)
    const uint32_t e = tid | (L << 8);
    uint16_t *dst = L <= 8 ? s_t1 + (code >> 8) : s_t2 + s_group[code >> 8] * 256u + (code & 0xFFu);
    const uint32_t n = L <= 8 ? 1u << (8 - L) : 1u << (16 - L);
    if (n >= 8) {
      const uint32_t e2 = e | (e << 16);
      uint4 *v = reinterpret_cast<uint4 *>(dst);
      for (uint32_t i = 0; i < n / 8; ++i) v[i] = make_uint4(e2, e2, e2, e2);
    } else {
      for (uint32_t i = 0; i < n; ++i) dst[i] = (uint16_t)e;
    }
  }
  __syncthreads();  // (valid prefix code: a group's high byte carries no short code)
  if (tid < 256 && s_group[tid]) s_t1[tid] = (uint16_t)s_group[tid];
  __syncthreads();
  TAB_STAMP(8);
  if (blockIdx.x == 0) {
    // out: T1, T2 over its whole capacity (zero past the used subtables)
    if (((uintptr_t)t1 & 15u) == 0) {
      if (tid < 32) reinterpret_cast<uint4 *>(t1)[tid] = reinterpret_cast<const uint4 *>(s_t1)[tid];
    } else if (tid < 256) {
      t1[tid] = s_t1[tid];
    }
    if (((uintptr_t)t2 & 15u) == 0) {
      uint4 *v = reinterpret_cast<uint4 *>(t2);
      for (uint32_t i = tid; i < kT2Vec; i += blockDim.x) v[i] = i < used_vec ? s_t2v[i] : make_uint4(0, 0, 0, 0);
    } else {
      for (uint32_t i = tid; i < (uint32_t)MH_TABLE2_MAX_ENTRIES; i += blockDim.x) t2[i] = i < used_vec * 8 ? s_t2[i] : 0;
    }
    if (tid == 0) {
      *t2_entries = bad ? 256u : (s_ngroups + 1u) * 256u;
      if (status) *status = bad ? ((s_bad & 1u) ? MH_ERR_CODE_TOO_LONG : MH_ERR_TABLE) : MH_OK;
    }
    if (lut && tid < 4) {  // [longest code, shortest code, flat8, 0] (mh_lut.hpp)
      // canonical codes: all 256 symbols at 8 bits is exactly the identity code c = symbol c
      const uint32_t flat = !bad && s_wcnt[0][8] + s_wcnt[1][8] + s_wcnt[2][8] + s_wcnt[3][8] == 256u;
      reinterpret_cast<uint32_t *>(lut + kMaxLenOff)[tid] = tid == 0 ? s_mx : tid == 1 ? s_mn : tid == 2 ? flat : 0u;
    }
  }
  if (!lut) return;
  // this workgroup's slice of the prepared entries: L1 | L2 | the 14-bit table
  uint32_t lmin = 0;  // shortest code length above 13 bits, 0 if none
  for (uint32_t l = 16; l > (uint32_t)kLutBits; --l)
    if (s_wcnt[0][l] + s_wcnt[1][l] + s_wcnt[2][l] + s_wcnt[3][l]) lmin = l;
  const uint32_t P0 = (!bad && lmin) ? (((s_first[lmin] << (16 - lmin)) & 0xFFFFu) >> kL2Bits)
                                     : (uint32_t)kL1Entries;
  const uint32_t nl2 = ((uint32_t)kL1Entries - P0) << kL2Bits;
  constexpr uint32_t kL2Region = (uint32_t)(kLutEntries - kL1Entries);
  constexpr uint32_t kAll = (uint32_t)kL1Entries + kL2Region + (uint32_t)kLut14Entries;
  const uint32_t per = (kAll + gridDim.x - 1) / gridDim.x;
  const uint32_t lo = blockIdx.x * per, hi = min(kAll, lo + per);
  uint16_t *out = reinterpret_cast<uint16_t *>(lut);
  uint16_t *out14 = reinterpret_cast<uint16_t *>(lut + kLut14Off);
  auto lookup = [&](uint32_t pat16) -> uint32_t {
    uint32_t e = s_t1[pat16 >> 8];
    if ((e >> 8) == 0) e = s_t2[(e & 0xFFu) * 256u + (pat16 & 0xFFu)];
    return e;
  };
  for (uint32_t v = lo + tid; v < hi; v += blockDim.x) {
    if (v < (uint32_t)kL1Entries) {
      const uint32_t p = v;
      uint32_t w;
      if (p >= P0) {
        const uint32_t sub = p - P0 + 1;
        w = sub < (uint32_t)kL2Subtables ? sub : 0u;
      } else {
        w = step_word(lookup(p << kL2Bits));
      }
      out[p] = (uint16_t)w;
    } else if (v < (uint32_t)kL1Entries + kL2Region) {
      const uint32_t i = v - (uint32_t)kL1Entries;  // L2 subtable 0 and the padding stay zero
      const uint32_t j = i - (1u << kL2Bits);
      const bool live = i >= (1u << kL2Bits) && j < nl2 && j < (uint32_t)(kL2Entries - (1 << kL2Bits));
      out[kL1Entries + i] = (uint16_t)(live ? step_word(lookup((P0 << kL2Bits) + j)) : 0u);
    } else {
      const uint32_t q = v - (uint32_t)kL1Entries - kL2Region;
      const uint32_t e = lookup(q << (16 - kLut14Bits));
      out14[q] = (uint16_t)((e >> 8) <= (uint32_t)kLut14Bits ? step_word(e) : 0u);
    }
  }
  __syncthreads();
  TAB_STAMP(15);
}

}  // namespace

extern "C" int mh_build_tables_device(const uint8_t *d_canon_header, mh_lookup_symbol *d_table1,
                                      mh_lookup_symbol *d_table2, uint32_t *d_table2_entries,
                                      uint16_t *d_lut, int32_t *d_status, void *stream) {
  if (!d_canon_header || !d_table1 || !d_table2 || !d_table2_entries) return MH_ERR_INVALID_ARG;
  if ((uintptr_t)d_lut & 15u) return MH_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(mh_build_tables_kernel, dim3(d_lut ? kTableGroups : 1), dim3(1024), 0, s, d_canon_header,
                     reinterpret_cast<uint16_t *>(d_table1), reinterpret_cast<uint16_t *>(d_table2),
                     d_table2_entries, d_status, reinterpret_cast<uint8_t *>(d_lut));
  return hipGetLastError() == hipSuccess ? MH_OK : MH_ERR_HIP;
}

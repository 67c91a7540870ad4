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
// range without ordering concerns. Headers that are not prefix codes (Kraft sum
// > 1) or hold a length > 16 are rejected with a status word.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "../../include/metalhuffman.h"

namespace {

__global__ void __launch_bounds__(1024) mh_build_tables_kernel(const uint8_t *canon, uint16_t *t1,
                                                               uint16_t *t2, uint32_t *t2_entries,
                                                               int32_t *status) {
  __shared__ uint32_t s_len[256], s_code[256], s_mark[256], s_group[256];
  __shared__ uint32_t s_cnt[17], s_first[17], s_kraft, s_bad, s_ngroups;
  const uint32_t tid = threadIdx.x;

  for (uint32_t i = tid; i < (uint32_t)MH_TABLE2_MAX_ENTRIES; i += blockDim.x) t2[i] = 0;
  if (tid < 256) {
    t1[tid] = 0;
    s_len[tid] = canon[tid];
    s_mark[tid] = 0;
  }
  if (tid < 17) s_cnt[tid] = 0;
  if (tid == 0) {
    s_kraft = 0;
    s_bad = 0;
  }
  __syncthreads();

  const uint32_t L = tid < 256 ? s_len[tid] : 0u;
  if (tid < 256 && L) {
    if (L > 16) {
      atomicOr(&s_bad, 1u);
    } else {
      atomicAdd(&s_cnt[L], 1u);
      atomicAdd(&s_kraft, 1u << (16 - L));
    }
  }
  __syncthreads();
  if (tid == 0) {
    // first code of each length: shift left across every length step
    uint32_t code = 0;
    for (uint32_t l = 1; l <= 16; ++l) {
      s_first[l] = code;
      code = (code + s_cnt[l]) << 1;
    }
    if (s_kraft > 65536u) s_bad |= 2u;
  }
  __syncthreads();
  if (s_bad) {
    if (tid == 0) {
      *t2_entries = 256;
      if (status) *status = (s_bad & 1u) ? MH_ERR_CODE_TOO_LONG : MH_ERR_TABLE;
    }
    return;
  }

  if (tid < 256 && L) {
    uint32_t rank = 0;  // symbols of the same length before this one
    for (uint32_t s = 0; s < tid; ++s) rank += s_len[s] == L ? 1u : 0u;
    const uint32_t code = ((s_first[L] + rank) << (16 - L)) & 0xFFFFu;
    s_code[tid] = code;
    if (L > 8) s_mark[code >> 8] = 1;
  }
  __syncthreads();
  if (tid < 256) {
    uint32_t g = 0;
    for (uint32_t h = 0; h < tid; ++h) g += s_mark[h];
    s_group[tid] = s_mark[tid] ? g + 1u : 0u;
    if (tid == 255) s_ngroups = g + s_mark[255];
  }
  __syncthreads();

  if (tid < 256 && L) {
    const uint32_t code = s_code[tid];
    const uint16_t e = (uint16_t)(tid | (L << 8));
    if (L <= 8) {
      for (uint32_t i = 0; i < (1u << (8 - L)); ++i) t1[(code >> 8) + i] = e;
    } else {
      uint16_t *sub = t2 + s_group[code >> 8] * 256u;
      for (uint32_t i = 0; i < (1u << (16 - L)); ++i) sub[(code & 0xFFu) + i] = e;
    }
  }
  __syncthreads();  // (valid prefix code: a group's high byte carries no short code)
  if (tid < 256 && s_group[tid]) t1[tid] = (uint16_t)s_group[tid];
  if (tid == 0) {
    *t2_entries = (s_ngroups + 1u) * 256u;
    if (status) *status = MH_OK;
  }
}

}  // namespace

extern "C" int mh_build_tables_device(const uint8_t *d_canon_header, mh_lookup_symbol *d_table1,
                                      mh_lookup_symbol *d_table2, uint32_t *d_table2_entries,
                                      uint16_t *d_lut, int32_t *d_status, void *stream) {
  if (!d_canon_header || !d_table1 || !d_table2 || !d_table2_entries) return MH_ERR_INVALID_ARG;
  if ((uintptr_t)d_lut & 15u) return MH_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(mh_build_tables_kernel, dim3(1), dim3(1024), 0, s, d_canon_header,
                     reinterpret_cast<uint16_t *>(d_table1), reinterpret_cast<uint16_t *>(d_table2),
                     d_table2_entries, d_status);
  if (hipGetLastError() != hipSuccess) return MH_ERR_HIP;
  // The prepared table reads T2 through its full (zero-padded) capacity.
  return d_lut ? mh_prepare_lut(d_table1, d_table2, MH_TABLE2_MAX_ENTRIES, d_lut, stream) : MH_OK;
}

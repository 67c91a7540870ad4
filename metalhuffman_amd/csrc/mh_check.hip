// mh_check.hip -- the decode contract's optional debug mode (SURVEY.md 8(b),
// "Errors"): walk every block exactly as the decoder does and report, per frame,
// what the reference would silently accept:
//   [0] zero-width lookups -- windows no code matches, the reference's {0, 0}
//       entry (T2 dummy subtable, HuffmanUtil.cpp:550-556); the decoder emits
//       `prev` again and does not advance (AAPLShaders.metal:258-262);
//   [1] T1 escapes past table2_entries (a subtable index > k; the reference
//       would read out of bounds, AAPLShaders.metal:159-170);
//   [2] blocks whose 64 codes do not end at the next block's offset (the
//       per-block offsets and the bitstream disagree; a frame's last block is
//       not checked, its end is not recorded);
//   [3] the first block (frame relative) with any of the above, or 0xFFFFFFFF.
// It never writes the raster and is not on the decode path's clock: one thread
// per block, tables read through the cache.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "../../include/metalhuffman.h"

namespace {

__global__ void __launch_bounds__(256) mh_check_init_kernel(uint32_t *report, uint32_t n_frames) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_frames * 4u) report[i] = (i & 3u) == 3u ? 0xFFFFFFFFu : 0u;
}

// 16-bit window at bit `pos` from 3 bytes (AAPLShaders.metal:137-155); bytes at
// or past `nbytes` read as zero (the decoder's buffer descriptors do the same).
__device__ __forceinline__ uint32_t window16(const uint8_t *c, uint64_t nbytes, uint64_t pos) {
  const uint64_t i = pos >> 3;
  const uint32_t m = (uint32_t)(pos & 7u);
  const uint32_t b0 = i < nbytes ? c[i] : 0u;
  const uint32_t b1 = i + 1 < nbytes ? c[i + 1] : 0u;
  const uint32_t b2 = i + 2 < nbytes ? c[i + 2] : 0u;
  return ((((b0 << 8) | b1) << 8 | b2) >> (8u - m)) & 0xFFFFu;
}

__global__ void __launch_bounds__(256) mh_check_kernel(const uint32_t *offsets, const uint8_t *codes,
                                                       const uint64_t *frame_off, uint64_t codes_bytes,
                                                       const uint16_t *t1, const uint16_t *t2,
                                                       uint32_t t2_entries, uint32_t nb,
                                                       uint32_t n_frames, uint32_t *report) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (uint64_t)nb * n_frames) return;
  const uint32_t f = (uint32_t)(g / nb), b = (uint32_t)(g % nb);
  uint64_t base = 0, fbytes = codes_bytes;
  if (frame_off) {
    base = frame_off[f];
    fbytes = frame_off[f + 1] - base;
  }
  const uint8_t *c = codes + base;
  uint64_t pos = offsets[g];
  uint32_t zero_width = 0, bad_escape = 0;
  for (int k = 0; k < 64; ++k) {
    const uint32_t pat = window16(c, fbytes, pos);
    uint32_t e = t1[pat >> 8];
    if ((e >> 8) == 0) {
      const uint32_t idx = (e & 0xFFu) * 256u + (pat & 0xFFu);
      if (idx < t2_entries) {
        e = t2[idx];
      } else {
        ++bad_escape;
        e = 0;
      }
    }
    const uint32_t len = e >> 8;
    zero_width += len == 0 ? 1u : 0u;
    pos += len;
  }
  const uint32_t mismatch = (b + 1u < nb && pos != offsets[g + 1]) ? 1u : 0u;
  if (zero_width | bad_escape | mismatch) {
    uint32_t *r = report + 4u * f;
    if (zero_width) atomicAdd(&r[0], zero_width);
    if (bad_escape) atomicAdd(&r[1], bad_escape);
    if (mismatch) atomicAdd(&r[2], 1u);
    atomicMin(&r[3], b);
  }
}

}  // namespace

extern "C" int mh_check(const mh_frame *fr, uint32_t *d_report, void *stream) {
  if (!fr || !d_report || !fr->d_block_offsets || !fr->d_codes || !fr->d_table1 || !fr->d_table2)
    return MH_ERR_INVALID_ARG;
  if (fr->n_frames == 0 || (fr->n_frames > 1 && !fr->d_frame_code_offsets)) return MH_ERR_INVALID_ARG;
  const mh_dims &d = fr->dims;
  if (!d.width || !d.height || d.width > MH_MAX_DIM || d.height > MH_MAX_DIM ||
      d.block_width != (d.width + 7) / 8 || d.block_height != (d.height + 7) / 8)
    return MH_ERR_DIMS;
  if (fr->table2_entries < 256 || (fr->table2_entries % 256) != 0 ||
      fr->table2_entries > MH_TABLE2_MAX_ENTRIES)
    return MH_ERR_TABLE;
  if (((uintptr_t)d_report & 3u)) return MH_ERR_ALIGN;
  const uint32_t nb = d.block_width * d.block_height;
  const uint64_t total = (uint64_t)nb * fr->n_frames;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(mh_check_init_kernel, dim3((fr->n_frames * 4u + 255u) / 256u), dim3(256), 0, s,
                     d_report, fr->n_frames);
  hipLaunchKernelGGL(mh_check_kernel, dim3((uint32_t)((total + 255u) / 256u)), dim3(256), 0, s,
                     fr->d_block_offsets, fr->d_codes, fr->d_frame_code_offsets,
                     fr->codes_bytes, reinterpret_cast<const uint16_t *>(fr->d_table1),
                     reinterpret_cast<const uint16_t *>(fr->d_table2), fr->table2_entries, nb,
                     fr->n_frames, d_report);
  return hipGetLastError() == hipSuccess ? MH_OK : MH_ERR_HIP;
}

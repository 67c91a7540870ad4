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

#include <stdint.h>

#include "../../include/metalhuffman.h"

namespace {

#ifndef MH_MAX_WAVES
#define MH_MAX_WAVES 8
#endif
#ifndef MH_DIAG_BROADCAST_LUT   // diagnostic builds only: LUT index forced to 0 (wrong output)
#define MH_DIAG_BROADCAST_LUT 0
#endif
#ifndef MH_NT_STORE
#define MH_NT_STORE 1
#endif
constexpr int kLutBits = 13;                  // first-level index width
constexpr int kL1Entries = 1 << kLutBits;     // 8192 x u16
constexpr int kL2Bits = 16 - kLutBits;        // 3 more window bits for long codes
constexpr int kL2Subtables = 129;             // dummy + <=128 long-code prefixes
constexpr int kL2Entries = kL2Subtables << kL2Bits;      // 1032
constexpr int kLutEntries = kL1Entries + 1040;           // L1 + L2, padded to 16 B
constexpr int kLutBytes = kLutEntries * 2;               // 18464
constexpr int kStageBytes = 4352;             // per-wave LDS window (max tile span)
constexpr int kMaxWavesPerWG = MH_MAX_WAVES;
static_assert(kLutBytes % 16 == 0, "lut copy uses 16-byte chunks");
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
  uint32_t t2_entries;
  uint32_t w, h, bw, bh, nb;
  uint32_t tiles_per_frame, total_tiles;
  uint32_t n_groups;           // ceil(total_tiles / waves_per_wg)
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
//   L1[p] (p = 13-bit prefix): split_lookup(p << 3) when that code has <= 13 bits
//     or the window is invalid (entry 0 -> dummy subtable 0 -> {0,0}, as the
//     reference's dummy T2 subtable, HuffmanUtil.cpp:550-556); otherwise an
//     escape {sub, 0}. Canonical codes are ordered by length, so every code of
//     14-16 bits lies at or above the first such code's prefix P0 and the long
//     codes (<= 256 codes of >= 4 patterns) occupy at most 128 prefixes from P0.
//   L2[sub*8 + x] = split_lookup(((P0 + sub - 1) << 3) | x), sub >= 1.
template <class SyncFn>
__device__ void build_lut(const uint16_t *t1, const uint16_t *t2, uint32_t t2_entries,
                          uint16_t *lut, uint32_t *p0, uint32_t tid, uint32_t nthreads,
                          SyncFn sync) {
  if (tid == 0) *p0 = (uint32_t)kL1Entries;
  sync();
  for (uint32_t p = tid; p < (uint32_t)kL1Entries; p += nthreads) {
    const uint32_t e = split_lookup(t1, t2, t2_entries, p << kL2Bits);
    lut[p] = (uint16_t)e;
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
    lut[kL1Entries + (1 << kL2Bits) + i] = (uint16_t)split_lookup(t1, t2, t2_entries, (P0 << kL2Bits) + i);
  sync();
}

__global__ void __launch_bounds__(1024) mh_prepare_lut_kernel(const uint16_t *t1, const uint16_t *t2,
                                                              uint32_t t2_entries, uint16_t *lut) {
  __shared__ uint32_t p0;
  build_lut(t1, t2, t2_entries, lut, &p0, threadIdx.x, blockDim.x, [] { __syncthreads(); });
}

// Word sources for the bit cursor: big-endian dwords of the tile's code span.
struct LdsWords {
  const uint32_t *w;
  __device__ __forceinline__ uint32_t operator()(uint32_t i) const { return w[i]; }
};
struct GlobalWords {  // fallback when a tile's span exceeds the LDS window
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t base;
  __device__ __forceinline__ uint32_t operator()(uint32_t i) const {
    return bswap32(__builtin_amdgcn_raw_buffer_load_b32(rsrc, (int)(base + 4u * i), 0, 0));
  }
};

// byte-insert selectors for v_perm_b32: put S0.byte0 at byte J, keep S1's others
__device__ __forceinline__ constexpr uint32_t ins_sel(int j) {
  return j == 0 ? 0x03020104u : j == 1 ? 0x03020400u : j == 2 ? 0x03040100u : 0x04020100u;
}

__shared__ __attribute__((aligned(16))) uint16_t s_lut[kLutEntries];
__shared__ __attribute__((aligned(16))) uint8_t s_stage[kMaxWavesPerWG * kStageBytes];
__shared__ uint32_t s_p0;

// One lane decodes one 8x8 block: 64 serial steps of AAPLShaders.metal:241-268
// (cursor advance, delta fold); rows are stored as they complete.
template <bool kDelta, class Src>
__device__ __forceinline__ void decode_block(const Src &src, uint32_t p, uint32_t prev,
                                             bool store, uint8_t *dst, uint64_t pitch,
                                             uint32_t cols, uint32_t rows) {
  uint32_t wi = p >> 5;
  uint32_t sh = p & 31u;
  uint32_t hi = src(wi);
  uint32_t lo = src(wi + 1);
  wi += 2;
  uint32_t nw = src(wi);

  // window = next 32 bits of the block's stream; sh <= 47 keeps >= 16 valid.
#define MH_STEP(J, OW)                                                              \
  {                                                                                 \
    const uint32_t win = (uint32_t)(((((uint64_t)hi) << 32) | lo) << sh >> 32);     \
    uint32_t e = s_lut[MH_DIAG_BROADCAST_LUT ? 0u : (win >> (32 - kLutBits))];     \
    const bool esc = e < 256u;                                                      \
    if (__builtin_expect(__ballot(esc) != 0, 0)) {                                  \
      const uint32_t e2 = s_lut[kL1Entries + ((e & 0xFFu) << kL2Bits) +             \
                                ((win >> (32 - 16)) & ((1u << kL2Bits) - 1u))];     \
      e = esc ? e2 : e;                                                             \
    }                                                                               \
    sh += e >> 8;                                                                   \
    if (kDelta) {                                                                   \
      prev += e;                                                                    \
      OW = __builtin_amdgcn_perm(prev, OW, ins_sel(J));                             \
    } else {                                                                        \
      OW = __builtin_amdgcn_perm(e, OW, ins_sel(J));                                \
    }                                                                               \
  }
  // keep sh < 32 at the start of every symbol pair (each code is <= 16 bits)
#define MH_REFILL()                                                                 \
  {                                                                                 \
    const bool c = sh >= 32u;                                                       \
    hi = c ? lo : hi;                                                               \
    lo = c ? nw : lo;                                                               \
    sh &= 31u;                                                                      \
    wi += c ? 1u : 0u;                                                              \
    nw = src(wi);                                                                   \
  }

#pragma unroll 1
  for (uint32_t r = 0; r < 8; ++r) {
    uint32_t o0 = 0, o1 = 0;
    if (r) MH_REFILL();
    MH_STEP(0, o0);
    MH_STEP(1, o0);
    MH_REFILL();
    MH_STEP(2, o0);
    MH_STEP(3, o0);
    MH_REFILL();
    MH_STEP(0, o1);
    MH_STEP(1, o1);
    MH_REFILL();
    MH_STEP(2, o1);
    MH_STEP(3, o1);
    if (store && r < rows) {
      uint8_t *row = dst + (uint64_t)r * pitch;
      if (cols == 8) {
        if (MH_NT_STORE)
          __builtin_nontemporal_store(((uint64_t)o1 << 32) | o0, reinterpret_cast<uint64_t *>(row));
        else
          *reinterpret_cast<uint2 *>(row) = make_uint2(o0, o1);
      } else {  // right-edge block of a width that is not a multiple of 8 (crop)
        const uint64_t v = ((uint64_t)o1 << 32) | o0;
#pragma unroll
        for (uint32_t x = 0; x < 7; ++x)
          if (x < cols) row[x] = (uint8_t)(v >> (8 * x));
      }
    }
  }
#undef MH_STEP
#undef MH_REFILL
}

template <bool kDelta>
__global__ void __launch_bounds__(64 * kMaxWavesPerWG) mh_decode_kernel(const DecodeArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = blockDim.x >> 6;
  uint8_t *stage = s_stage + wave * kStageBytes;

  // ---- lookup table into LDS (shared by the workgroup) ----
  if (a.lut) {
    const v4u32 *src = reinterpret_cast<const v4u32 *>(a.lut);
    v4u32 *dstv = reinterpret_cast<v4u32 *>(s_lut);
    for (uint32_t i = threadIdx.x; i < (uint32_t)(kLutBytes / 16); i += blockDim.x) dstv[i] = src[i];
    __syncthreads();
  } else {
    build_lut(a.t1, a.t2, a.t2_entries, s_lut, &s_p0, threadIdx.x, blockDim.x,
              [] { __syncthreads(); });
  }

  for (uint32_t g = blockIdx.x; g < a.n_groups; g += gridDim.x) {
    const uint32_t tile = g * nwaves + wave;
    if (tile >= a.total_tiles) break;  // wave-uniform
    const uint32_t f = tile / a.tiles_per_frame;
    const uint32_t b0 = (tile - f * a.tiles_per_frame) * 64u;
    const uint32_t b = b0 + lane;
    const bool valid = b < a.nb;

    uint64_t fbeg = 0, fbytes = a.codes_bytes;
    if (a.frame_off) {
      fbeg = a.frame_off[f];
      fbytes = a.frame_off[f + 1] - fbeg;
    }
    const uint32_t *offs = a.offsets + (uint64_t)f * a.nb;
    const uint32_t off = valid ? offs[b] : 0u;
    const uint32_t sb = __builtin_amdgcn_readfirstlane(off);  // lane 0 is always valid
    const uint32_t fb32 = (uint32_t)(fbytes > 0xFFFFFFF0ull ? 0xFFFFFFF0ull : fbytes);
    const uint32_t eb = (b0 + 64u < a.nb) ? offs[b0 + 64u] : (fb32 > 0x1FFFFFFFu ? 0xFFFFFFFFu : fb32 * 8u);
    const uint32_t start = (sb >> 3) & ~15u;
    uint32_t end = (eb >> 3) + 24u;
    if (end > fb32 + 16u) end = fb32 + 16u;
    const uint32_t span = end > start ? ((end - start + 15u) & ~15u) : 0xFFFFFFFFu;

    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.codes + fbeg), (short)0, (int)fb32, 0x00020000);

    const uint32_t p = valid ? off - start * 8u : 0u;
    const uint32_t prev = (valid && a.block_init) ? a.block_init[(uint64_t)f * a.nb + b] : 0u;
    const uint32_t bx = b % a.bw, by = b / a.bw;
    const uint32_t cols = min(8u, a.w - min(a.w, bx * 8u));
    const uint32_t rows = min(8u, a.h - min(a.h, by * 8u));
    uint8_t *dst = a.out + (uint64_t)f * a.out_frame_stride + (uint64_t)by * 8u * a.out_pitch + bx * 8u;

    if (span <= (uint32_t)kStageBytes) {
      for (uint32_t c = lane; c * 16u < span; c += 64u) {
        v4u32 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(start + c * 16u), 0, 0);
        v.x = bswap32(v.x);
        v.y = bswap32(v.y);
        v.z = bswap32(v.z);
        v.w = bswap32(v.w);
        *reinterpret_cast<v4u32 *>(stage + c * 16u) = v;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      LdsWords src{reinterpret_cast<const uint32_t *>(stage)};
      decode_block<kDelta>(src, p, prev, valid, dst, a.out_pitch, cols, rows);
      // the next tile's staging writes stay behind this tile's reads
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
      GlobalWords src{rsrc, start};
      decode_block<kDelta>(src, p, prev, valid, dst, a.out_pitch, cols, rows);
    }
  }
}

int g_cu_count = 0;
int g_occ[2][kMaxWavesPerWG + 1];

int cu_count() {
  if (!g_cu_count) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
    g_cu_count = prop.multiProcessorCount;
  }
  return g_cu_count;
}

template <bool kDelta>
int occupancy(int nw) {
  int &o = g_occ[kDelta ? 1 : 0][nw];
  if (!o) {
    int blocks = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, mh_decode_kernel<kDelta>, nw * 64, 0) !=
            hipSuccess ||
        blocks < 1)
      blocks = 1;
    o = blocks;
  }
  return o;
}

template <bool kDelta>
int launch(const DecodeArgs &a0, hipStream_t s) {
  DecodeArgs a = a0;
  const int cus = cu_count();
  if (!cus) return MH_ERR_HIP;
  // Waves per workgroup: spread a small launch (one 2048x1536 frame = 768 tiles)
  // over every CU; 8-wave workgroups (3 per CU by LDS) for batches.
  uint32_t nw = (a.total_tiles + (uint32_t)cus - 1) / (uint32_t)cus;
  if (nw < 1) nw = 1;
  if (nw > (uint32_t)kMaxWavesPerWG) nw = kMaxWavesPerWG;
  a.n_groups = (a.total_tiles + nw - 1) / nw;
  const uint32_t resident = (uint32_t)(cus * occupancy<kDelta>((int)nw));
  const uint32_t grid = a.n_groups < resident ? a.n_groups : resident;
  hipLaunchKernelGGL(mh_decode_kernel<kDelta>, dim3(grid), dim3(nw * 64), 0, s, a);
  return hipGetLastError() == hipSuccess ? MH_OK : MH_ERR_HIP;
}

}  // namespace

extern "C" {

size_t mh_lut_bytes(void) { return (size_t)kLutBytes; }
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
                     reinterpret_cast<const uint16_t *>(d_table2), table2_entries, d_lut);
  return hipGetLastError() == hipSuccess ? MH_OK : MH_ERR_HIP;
}

int mh_decode(const mh_frame *fr, uint8_t *d_out, size_t out_pitch, size_t out_frame_stride,
              void *stream) {
  if (!fr || !d_out || !fr->d_block_offsets || !fr->d_codes || !fr->d_table1 || !fr->d_table2)
    return MH_ERR_INVALID_ARG;
  if (fr->n_frames == 0 || (fr->n_frames > 1 && !fr->d_frame_code_offsets)) return MH_ERR_INVALID_ARG;
  if (fr->flags & ~MH_FLAG_NO_DELTA) return MH_ERR_INVALID_ARG;
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
  if (out_pitch < d.width || (fr->n_frames > 1 && out_frame_stride < out_pitch * d.height))
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
  return (fr->flags & MH_FLAG_NO_DELTA) ? launch<false>(a, s) : launch<true>(a, s);
}

}  // extern "C"

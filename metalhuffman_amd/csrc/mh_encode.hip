// mh_encode.hip -- GPU encoder for 8-bit grayscale frames:
// the producer side of the path, byte-identical to mh_encode_frame (mh_host.cpp),
// which itself reproduces the reference encoder:
//   split + deltas   Shared/Util.m:233-323, Shared/AAPLRenderer.m:432-515 (eight lanes
//                    per 8x8 block, zero padding past W/H, optional init byte :449-473)
//   histogram        HuffmanEncoder.cpp:310-330 (symbol counts; LDS, then global atomics
//                    into kHistParts partial histograms, and per-tile counts)
//   code lengths     HuffmanEncoder.cpp:29-145 -- the reference's sorted node array with
//                    upper_bound insertion is the two-queue Huffman merge with ties going
//                    to the leaf queue, run in batched rounds; then canonical codes
//                    huff_util.hpp:94-193 and the code byte count
//   block offsets    HuffmanUtil.cpp:1103-1128 -- an exclusive prefix sum of the
//                    per-block code-length sums
//   bit packing      HuffmanEncoder.cpp:211-381 -- MSB-first, staged per workgroup in LDS
// Frames of <= kFusedMaxTiles tiles: two launches, enc_split_kernel (tiled) and
// enc_code_kernel (workgroup 0 = tree, the others = offsets + packing of one tile each).
// Larger frames: enc_split_kernel, enc_tree_kernel, enc_scan_kernel, enc_pack_kernel.
// mh_encode_frame_device_async never synchronises (header, code bytes and status are
// written to device memory); mh_encode_frame_device runs it and synchronises once at
// the end to return the header and the byte count on the host.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "../../include/metalhuffman.h"


namespace {

constexpr uint32_t kScanTile = 256;  // blocks per workgroup in the offsets scan
constexpr uint32_t kResultBytes = 512;  // mh_encode_frame_device: header, byte count, status
constexpr uint32_t kHistParts = 8;      // partial histograms the split workgroups add into
constexpr uint32_t kTotalBits = 17;     // meta[] slot of the frame's code bit count
constexpr uint32_t kFlag = 18;          // meta[] slot: the code table is published (fused path)
constexpr uint32_t kAbort = 19;         // meta[] slot: a packing workgroup gave up waiting (fused path)
constexpr uint32_t kGen = 22;           // meta[] slot: call generation of the fused path (table tags)
#ifndef MH_DIAG_SPIN_TICKS  // diagnostic builds only (tests/test_gpu_encode.py: forced timeout)
#define MH_DIAG_SPIN_TICKS 10000000
#endif
constexpr uint64_t kSpinTicks = MH_DIAG_SPIN_TICKS;  // a packer's wait limit: 100 ms of s_memrealtime (100 MHz)
constexpr uint32_t kCodeTile = 128;     // blocks per tile of the fused path (split + code kernels)
constexpr uint32_t kFusedMaxTiles = 512;  // frames up to this many tiles take the two-kernel path

#ifndef MH_DIAG_SPLIT_NO_HIST  // diagnostic builds only: the tiled split without its LDS histogram
#define MH_DIAG_SPLIT_NO_HIST 0  // atomics (wrong output; the split's time without them)
#endif
#ifndef MH_DIAG_PACK_NO_OR  // diagnostic builds only: the batched packer without its LDS code-word
#define MH_DIAG_PACK_NO_OR 0  // ORs (wrong output; the packer's time without them)
#endif
#ifndef MH_CODE_STAMPS  // diagnostic builds only: s_memrealtime phase stamps of enc_code_kernel
#define MH_CODE_STAMPS 0
#endif
#if MH_CODE_STAMPS
constexpr uint32_t kCodeStampWgs = 1024;
__device__ unsigned long long g_code_stamps[kCodeStampWgs * 8];
__device__ unsigned long long g_split_stamps[kCodeStampWgs * 8];
#define MH_SPLIT_STAMP(k) \
  if (threadIdx.x == 0 && blockIdx.x < kCodeStampWgs) g_split_stamps[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime();
#define MH_CODE_STAMP(wg, k) \
  if (threadIdx.x == 0 && (wg) < kCodeStampWgs) g_code_stamps[(wg) * 8 + (k)] = __builtin_amdgcn_s_memrealtime();
#else
#define MH_SPLIT_STAMP(k)
#define MH_CODE_STAMP(wg, k)
#endif
struct Workspace {  // carved out of the caller's workspace, 256-B aligned parts
  uint8_t *sym;       // nb * 64 block symbols
  uint32_t *blen;     // nb per-block bit lengths
  uint32_t *tsum;     // ceil(nb / kScanTile) tile sums (then tile offsets)
  uint64_t *hist;     // kHistParts x 256 partial counts
  uint32_t *table;    // 256 x (code_lj16 << 16 | len)
  uint64_t *meta;     // [codes_len, ok flag, .., [kTotalBits], [kFlag], [kAbort], [kGen]]
  uint16_t *tile_hist;  // fused path: ceil(nb / kCodeTile) x 256 symbol counts
};

constexpr uint64_t align256(uint64_t x) { return (x + 255) & ~255ull; }

// A workgroup barrier for LDS-only hand-offs: waits for this wave's LDS operations
// (lgkmcnt), not its global ones. __syncthreads()'s workgroup-scope fence also waits
// for every outstanding global load and store (vmcnt(0)) -- in the packers that put an
// HBM write round trip (the offsets, the code words) and any prefetch behind every
// barrier. Valid wherever the threads of a workgroup exchange data only through LDS.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

uint64_t carve(uint8_t *base, uint64_t nb, Workspace *w) {
  uint64_t o = 0;
  const uint64_t ntiles = (nb + kScanTile - 1) / kScanTile;
  if (w) w->sym = base + o;
  o += align256(nb * 64);
  if (w) w->blen = reinterpret_cast<uint32_t *>(base + o);
  o += align256(nb * 4);
  if (w) w->tsum = reinterpret_cast<uint32_t *>(base + o);
  o += align256(ntiles * 4);
  if (w) w->hist = reinterpret_cast<uint64_t *>(base + o);
  o += align256(kHistParts * 256 * 8);
  if (w) w->table = reinterpret_cast<uint32_t *>(base + o);
  o += align256(256 * 4);
  if (w) w->meta = reinterpret_cast<uint64_t *>(base + o);
  o += align256((kGen + 1) * 8);
  // hist, table and meta are contiguous: the per-call state a caller without
  // MH_ENCODE_WORKSPACE_ZEROED gets zeroed by one memset (mh_encode_frame_device_async)
  const uint64_t ncode = (nb + kCodeTile - 1) / kCodeTile;
  if (w) w->tile_hist = reinterpret_cast<uint16_t *>(base + o);  // u16 counts per code tile
  o += align256(ncode * 256 * 2);
  return o;
}

// Eight lanes per block, one 8-pixel block row each (lane = 8 * block + row), so a
// wave reads 8 image rows x 64 contiguous bytes and writes 512 contiguous symbol
// bytes. Pixels -> symbols (block order, row-major inside the block, zero past the
// frame edge), per-block deltas in SWAR with the previous pixel from the lane one
// row up, histogram into 16 replicated LDS copies (BigBridge-like deltas are mostly
// one symbol; one copy would serialise every atomic on it). Grid-stride over groups
// of 32 blocks; one global atomic per used bin per workgroup.
constexpr uint32_t kHistCopies = 16;  // 8: no faster, 32: 58 % slower (profiles/r04_v4_encoder_batch_ab.txt)
constexpr uint32_t kSplitBatch = 8;   // groups of 32 blocks whose rows a split workgroup loads at once
constexpr uint32_t kSplitWgs = 256;   // split workgroups (four-kernel path): one global atomic per used bin each

// Buffer descriptor from wave-uniform inputs (readfirstlane, so buffer ops need no
// waterfall loop); offsets past `bytes` are dropped by the hardware.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t enc_rsrc(const void *base, uint64_t bytes) {
  const uint64_t p = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
  const uint32_t n = (uint32_t)(bytes < 0x7FFFFFF0ull ? bytes : 0x7FFFFFF0ull);
  return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(n), 0x00020000);
}
constexpr uint32_t kOob = 0x80000000u;  // a buffer offset past every descriptor's range: dropped

// Row r (8 pixels, little-endian in a u64) of 8x8 block b, zero past the frame edge
// (Util.m:256-318: zero-filled blocks, row-major inside a block).
__device__ __forceinline__ uint64_t block_row(const uint8_t *gray, uint32_t W, uint32_t H, uint32_t bw,
                                              uint64_t nb, uint32_t vec, uint64_t b, uint32_t r) {
  if (b >= nb) return 0;
  // a frame has < 2^26 blocks (65535^2 / 64): 32-bit division (a 64-bit one is a long
  // software sequence per lane)
  const uint32_t b32 = (uint32_t)b, bx = b32 % bw, y = (b32 / bw) * 8 + r;
  if (y >= H) return 0;
  const uint8_t *row = gray + (uint64_t)y * W + bx * 8u;
  if (vec) return *reinterpret_cast<const uint64_t *>(row);  // W % 8 == 0, 8-byte aligned frame
  uint64_t q = 0;
  for (uint32_t c = 0; c < 8; ++c)
    if (bx * 8u + c < W) q |= (uint64_t)row[c] << (8 * c);
  return q;
}

// The 8 symbols of a block row from its pixels q (lane = 8 * block + r, all lanes
// converged): per-block deltas (AAPLRenderer.m:432-515) in SWAR, the previous pixel of
// row r > 0 being the last pixel of row r - 1, taken from the lane below by DPP
// row_shr:1 (row 0's first delta is against 0); with the init byte
// (AAPLRenderer.m:449-473) the block's first delta moves out and its symbol is 0.
__device__ __forceinline__ uint64_t row_symbols(uint64_t q, uint32_t r, bool delta, bool init_byte,
                                                uint32_t *first) {
  uint64_t v = q;
  *first = 0;
  if (delta) {
    const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(q >> 56), 0x111, 0xF, 0xF, false);
    const uint64_t p = (q << 8) | (r ? up : 0u);
    constexpr uint64_t kH = 0x8080808080808080ull;
    v = ((q | kH) - (p & ~kH)) ^ ((q ^ ~p) & kH);  // bytewise q - p
    if (init_byte && r == 0) {
      *first = (uint32_t)v & 0xFFu;
      v &= ~0xFFull;
    }
  }
  return v;
}

// Tiled mode (tile_hist != null, the fused and batched paths): workgroup t owns the
// kCodeTile blocks of tile t (kCodeTile / 32 consecutive groups, loaded at once) and
// stores the tile's symbol counts in tile_hist[t]; with meta (the fused path) its
// workgroup 0 re-arms the code kernel's table flag. Batched frames: workgroup
// f * ncode + t is tile t of frame f (gray + f * gray_stride; per-frame block_init,
// hist and tile_hist slices).
constexpr uint32_t kTileGroups = kCodeTile / 32;
static_assert(kTileGroups <= kSplitBatch && kCodeTile % 32 == 0, "a split workgroup's batch covers a code tile");
// Blocks per tile of the batched path (split workgroup, tree tile counts, packer wave).
// 256 (round 5) halves round 4's per-tile records (counts, offsets, last-block symbols)
// that the split writes and the trees read: 64 BigBridge shuffles per call, 571 -> 557 MB
// of HBM traffic and 3.02-3.07 -> 2.88-2.93 us per frame (profiles/r05_encoder_batch_ab.txt).
// (128 and 512 measured beside it: the same file.)
constexpr uint32_t kBatchTile = 256;
static_assert(kBatchTile / 32 <= 2 * kSplitBatch && kBatchTile % 32 == 0 && kBatchTile * 64 < 65536,
              "a split workgroup loads a batch tile's rows at once; u16 tile counts");

// Row r of this lane's block (32 g + lane / 8) of group g as ONE unconditional buffer
// load (kVec: 8 bytes; else 8 byte loads), zero past the frame: a fixed count of loads
// per lane, so several groups' loads stay in flight together (a load under a branch
// makes the compiler wait for it at the join). The descriptor starts at the group's
// first block row (uniform), so offsets stay 32-bit for any frame size.
template <bool kVec>
__device__ __forceinline__ uint64_t group_row(const uint8_t *gray, uint32_t W, uint32_t H, uint32_t bw, uint64_t nb,
                                              uint64_t g, uint32_t r) {
  const uint32_t k = threadIdx.x >> 3;
  const uint64_t gb = g * 32;
  const uint32_t gb32 = (uint32_t)(gb < nb ? gb : nb);  // nb < 2^26
  const uint32_t by0 = gb32 / bw;                       // uniform
  uint32_t bx = gb32 - by0 * bw + k, by = by0;
  if (bw >= 32) {
    if (bx >= bw) {  // a group spans at most two block rows
      bx -= bw;
      ++by;
    }
  } else {
    by += bx / bw;
    bx %= bw;
  }
  const uint32_t y0 = by0 * 8u, y = by * 8u + r;
  const bool in = gb + k < nb && y < H;
  const __amdgpu_buffer_rsrc_t rg = enc_rsrc(gray + (uint64_t)y0 * W, y0 < H ? (uint64_t)(H - y0) * W : 0ull);
  if constexpr (kVec) {
    typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));
    const v2u32 v = __builtin_amdgcn_raw_buffer_load_b64(rg, (int)(in ? (y - y0) * W + bx * 8u : kOob), 0, 0);
    return ((uint64_t)v.y << 32) | v.x;
  } else {
    uint64_t q = 0;
#pragma unroll
    for (uint32_t c = 0; c < 8; ++c)
      q |= (uint64_t)__builtin_amdgcn_raw_buffer_load_b8(rg, (int)(in && bx * 8u + c < W ? (y - y0) * W + bx * 8u + c : kOob),
                                                         0, 0) << (8 * c);
    return q;
  }
}

// The tiled split's rows: lane k's blocks tb + k + 32 u (u < N) of the tile starting at
// block tb, row r, from one descriptor at the tile's first block row. The tile's
// coordinates are uniform (one scalar division); a lane's block wraps into the next
// block row at most once when the frame is >= kCodeTile blocks wide.
template <bool kVec, uint32_t N, uint32_t kTile>
__device__ __forceinline__ void tile_rows(const uint8_t *gray, uint32_t W, uint32_t H, uint32_t bw, uint64_t nb,
                                          uint32_t tb, uint32_t r, uint64_t (&q)[N]) {
  // no 64-bit compares and no per-load v_mul_lo (quarter rate): 32-bit block indices
  // (nb < 2^26), the row offset r * W once, a wrapped block adds 8 W
  const uint32_t k = threadIdx.x >> 3, nb32 = (uint32_t)nb;
  const uint32_t tby = tb / bw, tbx = tb - tby * bw;
  const uint32_t y0 = tby * 8u, hrem = H - y0, w8 = 8u * W;
  const __amdgpu_buffer_rsrc_t rg = enc_rsrc(gray + (uint64_t)y0 * W, (uint64_t)hrem * W);
  uint32_t rowoff = r * W;
  asm volatile("" : "+v"(rowoff));  // kept as is (else folded back into (dy + r) * W per load)
#pragma unroll
  for (uint32_t u = 0; u < N; ++u) {
    uint32_t bx = tbx + k + 32u * u, dy = 0, doff = 0;
    if (bw >= kTile) {
      const bool wrap = bx >= bw;
      bx = wrap ? bx - bw : bx;
      dy = wrap ? 8u : 0u;
      doff = wrap ? w8 : 0u;
    } else {
      const uint32_t d = bx / bw;
      bx -= d * bw;
      dy = d * 8u;
      doff = dy * W;
    }
    const bool in = tb + k + 32u * u < nb32 && dy + r < hrem;
    const uint32_t off = doff + rowoff + bx * 8u;
    if constexpr (kVec) {
      typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));
      const v2u32 v = __builtin_amdgcn_raw_buffer_load_b64(rg, (int)(in ? off : kOob), 0, 0);
      q[u] = ((uint64_t)v.y << 32) | v.x;
    } else {
      uint64_t x = 0;
#pragma unroll
      for (uint32_t c = 0; c < 8; ++c)
        x |= (uint64_t)__builtin_amdgcn_raw_buffer_load_b8(rg, (int)(in && bx * 8u + c < W ? off + c : kOob), 0, 0)
             << (8 * c);
      q[u] = x;
    }
  }
}

template <bool kVec, bool kTiled, uint32_t kTile = kCodeTile>
__global__ void __launch_bounds__(256) enc_split_kernel(const uint8_t *gray, uint32_t W, uint32_t H,
                                                        uint32_t bw, uint64_t nb, uint32_t flags,
                                                        uint8_t *sym, uint8_t *block_init,
                                                        uint64_t *hist, uint16_t *tile_hist, uint64_t *meta,
                                                        uint32_t ncode, uint64_t gray_stride,
                                                        uint64_t *tile_tail) {
  constexpr bool tiled = kTiled;
  uint32_t wg = blockIdx.x;  // tiled: this frame's tile
  if (tiled) {
    const uint32_t f = blockIdx.x / ncode;
    wg = blockIdx.x - f * ncode;
    gray += f * gray_stride;
    if (block_init) block_init += (uint64_t)f * nb;
    if (hist) hist += (uint64_t)f * kHistParts * 256;
    tile_hist += (uint64_t)f * ncode * 256;
    if (tile_tail) tile_tail += (uint64_t)f * ncode * 8;
  }
  if (tiled && meta && blockIdx.x == 0 && threadIdx.x == 0) {  // the code kernel runs after this one
    meta[kFlag] = 0;
    meta[kAbort] = 0;
    meta[kGen] += 1;  // a new tag for the code table words (table_tag)
  }
  MH_SPLIT_STAMP(0)
  __shared__ __attribute__((aligned(16))) uint32_t h[256 * kHistCopies];
  // the histogram is cleared behind the first batch's loads (their HBM round trip
  // covers it), before any atomic: 16-byte writes, consecutive per lane (no conflicts)
  bool cleared = false;
  const auto clear_hist = [&]() {
    typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (uint32_t i = 0; i < kHistCopies / 4; ++i) reinterpret_cast<v4u32 *>(h)[threadIdx.x + 256u * i] = v4u32{0u, 0u, 0u, 0u};
    lds_barrier();
    cleared = true;
  };
  const uint32_t r = threadIdx.x & 7u;
  const uint32_t copy = threadIdx.x % kHistCopies;
  const bool delta = !(flags & MH_FLAG_NO_DELTA);
  // block_init: buffer stores (lanes without a byte out of range)
  const __amdgpu_buffer_rsrc_t rinit = enc_rsrc(block_init, block_init ? nb : 0ull);
  // one group of 32 blocks: deltas, init bytes, symbols out (four-kernel path; the
  // fused path's packer re-derives them from the pixels), histogram
  // one group of 32 blocks (four-kernel path): deltas, init bytes, symbols out, histogram
  auto process = [&](uint64_t g, uint64_t q) {
    const uint64_t b = g * 32 + (threadIdx.x >> 3);
    const bool on = b < nb;
    uint32_t first;
    const uint64_t v = row_symbols(q, r, delta, block_init != nullptr, &first);
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)first, rinit, (int)(r == 0 && on ? (uint32_t)b : kOob), 0, 0);
    if (on) {
      if (sym) reinterpret_cast<uint64_t *>(sym + b * 64)[r] = v;  // large frames: 64-bit offsets
      for (int j = 0; j < 8; ++j) atomicAdd(&h[((uint32_t)(v >> (8 * j)) & 0xFFu) * kHistCopies + copy], 1u);
    }
  };
  const uint64_t ngroups = (nb + 31) / 32;
  constexpr uint32_t kGroups = kTile / 32;  // tiled: groups of 32 blocks per tile
  if constexpr (kTiled) {
    // One tile: its kGroups groups' rows loaded at once (8 bytes per lane in flight would
    // leave the read latency-bound), then each group's deltas and histogram. The init
    // bytes are stored only when the format has them (a uniform branch: no dead store per
    // row), and the tile's last block's symbols (batched path, tile_tail) once at the end.
    const uint32_t nb32 = (uint32_t)nb, tb = wg * kTile;
    uint64_t q[kGroups];
    tile_rows<kVec, kGroups, kTile>(gray, W, H, bw, nb, tb, r, q);
    clear_hist();
#if MH_CODE_STAMPS
    __builtin_amdgcn_s_waitcnt(0);
    MH_SPLIT_STAMP(1)
#endif
    uint64_t vlast = 0;
#pragma unroll
    for (uint32_t u = 0; u < kGroups; ++u) {
      const uint32_t b = tb + 32u * u + (threadIdx.x >> 3);
      uint32_t first;
      const uint64_t v = row_symbols(q[u], r, delta, block_init != nullptr, &first);
      if (block_init)  // kernel-uniform
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)first, rinit, (int)(r == 0 && b < nb32 ? b : kOob), 0, 0);
      if (!MH_DIAG_SPLIT_NO_HIST && b < nb32)
        for (int j = 0; j < 8; ++j) atomicAdd(&h[((uint32_t)(v >> (8 * j)) & 0xFFu) * kHistCopies + copy], 1u);
      vlast = v;
    }
    // the tile's last block (lanes 248-255 of group kGroups - 1): its symbols for the next
    // tile's packer, whose first code word starts with this block's last bits -- 64 B per
    // tile instead of the packer re-reading the block's eight pixel rows (eight 128-B lines)
    if (tile_tail && threadIdx.x >= 248u && tb + kTile - 1u < nb32) tile_tail[(uint64_t)wg * 8u + r] = vlast;
  } else {
    // grid-stride over groups, kSplitBatch groups' rows loaded before any is processed
    // (32-bit group indices: a frame has < 2^26 blocks, < 2^21 groups)
    const uint32_t ng32 = (uint32_t)ngroups, gdim = gridDim.x, gstride = kSplitBatch * gdim;
    for (uint32_t g0 = blockIdx.x; g0 < ng32; g0 += gstride) {
      uint64_t q[kSplitBatch];
#pragma unroll
      for (uint32_t u = 0; u < kSplitBatch; ++u) q[u] = group_row<kVec>(gray, W, H, bw, nb, g0 + u * gdim, r);
      if (!cleared) clear_hist();  // workgroup-uniform
#pragma unroll
      for (uint32_t u = 0; u < kSplitBatch; ++u) {
        const uint32_t g = g0 + u * gdim;
        if (g < ng32) process(g, q[u]);
      }
    }
  }
  MH_SPLIT_STAMP(2)
  if (!cleared) clear_hist();  // no group at all
  lds_barrier();
  uint32_t c = 0;
  for (uint32_t k = 0; k < kHistCopies; ++k) c += h[threadIdx.x * kHistCopies + ((k + threadIdx.x) % kHistCopies)];
  if (tiled) tile_hist[(uint64_t)wg * 256 + threadIdx.x] = (uint16_t)c;  // <= kTile * 64
  MH_SPLIT_STAMP(3)
  // kHistParts partial histograms (workgroups round-robin over them, as over the
  // XCDs): one address per bin would serialise every workgroup's atomic on it
  // (the batched path passes no hist: its tree kernel sums the tile counts itself)
  if (c && hist) atomicAdd((unsigned long long *)&hist[(wg % kHistParts) * 256 + threadIdx.x], (unsigned long long)c);
#if MH_CODE_STAMPS
  __builtin_amdgcn_s_waitcnt(0);
  MH_SPLIT_STAMP(4)
#endif
}


// Value of lane (lane ^ D) (64-lane wave): permlane32_swap for 32, ds_swizzle's xor
// mode for 16 and 4, DPP (row rotate by 8, quad permutes) for 8, 2, 1.
template <uint32_t D>
__device__ __forceinline__ uint32_t xor_partner(uint32_t lane, uint32_t v) {
  if constexpr (D == 32 || D == 16) {
    // the swap leaves lane ^ D's value in the first result for the upper lane of
    // each pair, in the second for the lower
    const auto r = D == 32 ? __builtin_amdgcn_permlane32_swap(v, v, false, false)
                           : __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (lane & D) ? r[0] : r[1];
  } else if constexpr (D == 8) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128 /* row_ror:8 */, 0xF, 0xF, true);
  } else if constexpr (D == 4) {  // row_half_mirror (i -> 7 - i) then reverse within quads
    const int m = __builtin_amdgcn_mov_dpp((int)v, 0x141 /* row_half_mirror */, 0xF, 0xF, true);
    return (uint32_t)__builtin_amdgcn_mov_dpp(m, 0x1B /* quad_perm [3,2,1,0] */, 0xF, 0xF, true);
  } else if constexpr (D == 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E /* quad_perm [2,3,0,1] */, 0xF, 0xF, true);
  } else {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1 /* quad_perm [1,0,3,2] */, 0xF, 0xF, true);
  }
}

// One half-cleaner stage of an ascending bitonic sort over the wave: the lower lane
// of each (lane, lane ^ D) pair keeps the smaller key, the upper the larger.
template <uint32_t D>
__device__ __forceinline__ void bitonic_stage(uint32_t lane, uint64_t &key) {
  const uint64_t p = ((uint64_t)xor_partner<D>(lane, (uint32_t)(key >> 32)) << 32) |
                     xor_partner<D>(lane, (uint32_t)key);
  const bool take = (p < key) != ((lane & D) != 0u);  // keys are distinct
  key = take ? p : key;
}

// ... on 32-bit keys (frames of < 2^22 symbols, see tree_body). Keys are distinct, so
// the lower lane keeps min(key, partner) and the upper one the max: v_min / v_max and
// one select on a lane-constant mask (no compare -> VCC -> select chain). The swap
// stages (D = 32, 16) take min / max straight from the two permlane outputs: each lane
// holds its own key in one and its partner's in the other.
template <uint32_t D>
__device__ __forceinline__ void bitonic_stage32(uint32_t lane, uint32_t &key) {
  uint32_t a, b;
  if constexpr (D == 32 || D == 16) {
    const auto r = D == 32 ? __builtin_amdgcn_permlane32_swap(key, key, false, false)
                           : __builtin_amdgcn_permlane16_swap(key, key, false, false);
    a = r[0];
    b = r[1];
  } else {
    a = key;
    b = xor_partner<D>(lane, key);
  }
  key = (lane & D) ? max(a, b) : min(a, b);
}

// Ascending bitonic sort of one key per lane over the wave (21 compare-exchange stages
// of size K, distance J; duplicates allowed): min / max plus one lane-constant select.
template <uint32_t K, uint32_t J>
__device__ __forceinline__ void sort_stage(uint32_t lane, uint32_t &key) {
  uint32_t a, b;
  if constexpr (J == 32 || J == 16) {  // each lane gets its own key in one output, its partner's in the other
    const auto r = J == 32 ? __builtin_amdgcn_permlane32_swap(key, key, false, false)
                           : __builtin_amdgcn_permlane16_swap(key, key, false, false);
    a = r[0];
    b = r[1];
  } else {
    a = key;
    b = xor_partner<J>(lane, key);
  }
  const bool up = K == 64 || (lane & K) == 0u;
  key = (((lane & J) == 0u) == up) ? min(a, b) : max(a, b);
}
template <uint32_t K, uint32_t J>
__device__ __forceinline__ void sort_merge(uint32_t lane, uint32_t &key) {
  sort_stage<K, J>(lane, key);
  if constexpr (J > 1) sort_merge<K, J / 2>(lane, key);
}
template <uint32_t K = 2>
__device__ __forceinline__ void wave_sort64(uint32_t lane, uint32_t &key) {
  sort_merge<K, K / 2>(lane, key);
  if constexpr (K < 64) wave_sort64<K * 2>(lane, key);
}

// The fused paths' call tag (1..255) in the code table words: from meta[kGen], which
// the split kernel (two-launch path) or the last workgroup of the previous launch
// (one-launch path) advances once per call.
__device__ __forceinline__ uint32_t table_tag(const uint64_t *meta) {
  return (__hip_atomic_load(reinterpret_cast<const uint32_t *>(&meta[kGen]), __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_AGENT) % 255u) + 1u;
}

// A packing workgroup's wait for the code table: threads 0-255 poll their own word
// until it carries this call's tag, then keep code | length in `tab`. Returns 1 (table
// in tab), 2 (a rejected frame: the tree set the bad bit) or 3 (timed out).
__device__ __forceinline__ uint32_t wait_table(const uint32_t *table, const uint64_t *meta, uint32_t *tab,
                                               uint32_t sleep_after) {
  const uint32_t tid = threadIdx.x;
  bool timeout = false, bad = false;
  if (tid < 256) {
    const uint32_t tag = table_tag(meta);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t w;
    uint32_t polls = 0;
    while (((w = __hip_atomic_load(&table[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 8 & 0xFFu) != tag) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {  // exit condition: never hang
        timeout = true;
        break;
      }
      if (++polls > sleep_after) __builtin_amdgcn_s_sleep(8);
      else __builtin_amdgcn_s_sleep(1);
    }
    tab[tid] = w & 0xFFFF001Fu;  // code (left-justified, 16 bits) << 16 | length
    bad = (w & 0x80u) != 0u;
  }
  const bool any_timeout = __syncthreads_or(timeout) != 0;
  const bool any_bad = __syncthreads_or(bad) != 0;
  return any_timeout ? 3u : any_bad ? 2u : 1u;
}

// One 256-thread workgroup: the reference's Huffman tree (HuffmanEncoder.cpp:29-145)
// from the 256 counts. The reference keeps every node in one array sorted by weight,
// inserts at upper_bound (a new node goes after all nodes of equal weight) and merges
// the two front-most entries. Leaves enter first, in symbol order, so they sit sorted
// by (weight, symbol); merged weights never decrease, so internal nodes sit in
// creation order after every leaf of equal weight. That is the two-queue merge
// (sorted leaves, internal nodes in creation order) taking the leaf on a tie: the
// same tree. The merge runs in rounds of up to 32 merges on one wave (see below);
// leaf ranks, depths (pointer jumping over the parent links) and canonical ranks
// (ballots) are parallel. Then
// the canonical codes
// (huff_util.hpp:94-193), the code table, the code byte count and the status
// (mh_code_lengths' errors, the caller's capacity).
constexpr uint32_t kTreeThreads = 1024;  // 4 per symbol in the ranking; 256 (one per symbol) elsewhere

// kFused: workgroup 0 of enc_code_kernel -- the table goes out as agent-scope
// (write-through) stores and meta[kFlag] publishes it to the packing workgroups.
// nsym: the frame's symbol count (64 per block). Below 2^22 - 1 every weight --
// root included -- fits 22 bits, and the ranking and merge keys fit 32 bits.
template <bool kFused>
// Returns, to the 256 symbol threads, symbol tid's table entry (code_lj16 << 16 | len;
// 0 for an absent symbol) with bit 7 set when the frame is rejected; the other
// threads return 0 early (before the symbol threads' last barriers).
// counts (optional): the 256 symbol counts already in LDS (the batched path sums its
// tile counts itself); otherwise they are the sum of hist's kHistParts partial
// histograms, which are left zeroed.
__device__ __forceinline__ uint32_t tree_body(uint64_t *hist, uint8_t *canon_out, uint32_t *table, uint64_t *meta,
                                          uint64_t *codes_len_out, uint64_t codes_cap, int32_t *status,
                                          uint64_t nsym, const uint32_t *counts = nullptr) {
  constexpr uint32_t kEnd = 0xFFFFFFFFu;  // empty queue slot
  constexpr uint32_t kW32End = (1u << 22) - 1u;  // 32-bit merge keys: an empty slot's weight
  const bool k32 = nsym < (uint64_t)kW32End;
  __shared__ uint32_t s_lw[384], s_iw[384];  // queues padded with kEnd
  __shared__ __attribute__((aligned(16))) uint64_t s_key[256];
  __shared__ __attribute__((aligned(16))) uint32_t s_key32[256];
  __shared__ uint32_t s_leaf_sym[256], s_len[256], s_par[2][512], s_dep[2][512];
  __shared__ uint32_t s_wcnt[4][17], s_first[17], s_n, s_bad;
  __shared__ uint32_t s_below[4][256];
  __shared__ unsigned long long s_total;
  const uint32_t tid = threadIdx.x;
  const bool sym_thread = tid < 256u;  // thread tid < 256 owns symbol tid
  // this call's table tag: meta[kGen] does not change during the launch, so its L2
  // round trip overlaps the histogram loads instead of preceding the publication
  const uint32_t tag = kFused && sym_thread ? table_tag(meta) : 0u;
  uint64_t f = 0;
  if (sym_thread && counts) {
    f = counts[tid];
  } else if (sym_thread) {
#pragma unroll
    for (uint32_t k = 0; k < kHistParts; ++k) f += hist[k * 256 + tid];
    // leave the histogram zeroed for the next frame's split (MH_ENCODE_WORKSPACE_ZEROED)
#pragma unroll
    for (uint32_t k = 0; k < kHistParts; ++k) hist[k * 256 + tid] = 0;
  }
  if (sym_thread) {
    s_len[tid] = 0;
    s_lw[tid] = kEnd;
    s_iw[tid] = kEnd;
  }
  if (tid < 128) s_lw[256 + tid] = s_iw[256 + tid] = kEnd;
  if (tid == 0) {
    s_n = 0;
    s_bad = 0;
    s_total = 0;
  }
  __syncthreads();
  {
    // rank of this leaf in (weight, symbol) order: count the smaller keys among all
    // 256 (16-byte broadcast reads, one 64-bit compare per key). Absent symbols
    // have key 0, below every present one: subtract their count afterwards.
    // Four threads per symbol, a quarter of the keys each (the compares are VALU
    // issue-bound: one wave per SIMD took 6 K clocks for all 256).
    const uint32_t ks = tid & 255u, part = tid >> 8;
    uint32_t below = 0, present;
    if (k32) {  // counts < 2^22: (count << 8 | symbol) fits 32 bits
      // The four symbol waves sort their 64 keys in registers (bitonic), then thread
      // (part, q) counts the keys of run `part` below sorted element q by binary search
      // (7 dependent LDS reads); q's rank is the sum over the four runs.
      uint32_t key = f ? (uint32_t)(f << 8) | tid : 0u;
      present = (uint32_t)__syncthreads_count(f != 0);
      if (sym_thread) {
        wave_sort64(tid & 63u, key);
        s_key32[tid] = key;
      }
      __syncthreads();
      const uint32_t kq = s_key32[ks];
      if (part == (ks >> 6)) {
        below = ks & 63u;  // its place in its own run (present keys are distinct)
      } else {
        const uint32_t *run = s_key32 + 64u * part;
#pragma unroll
        for (uint32_t step = 64; step; step >>= 1)
          if (below + step <= 64u && run[below + step - 1u] < kq) below += step;
      }
      s_below[part][ks] = below;
      __syncthreads();
      if (sym_thread) {
        const uint32_t k = s_key32[tid];  // sorted element tid
        if (k) {
          const uint32_t rank = s_below[0][tid] + s_below[1][tid] + s_below[2][tid] + s_below[3][tid] - (256u - present);
          s_leaf_sym[rank] = k & 0xFFu;
          s_lw[rank] = k >> 8;
        }
      }
    } else {
      if (sym_thread) s_key[tid] = f ? (f << 8) | tid : 0;
      present = (uint32_t)__syncthreads_count(f != 0);
      const uint64_t key = s_key[ks];
      const ulonglong2 *kv = reinterpret_cast<const ulonglong2 *>(s_key) + part * 32u;
#pragma unroll 16
      for (uint32_t t = 0; t < 32; ++t) {  // same address across the wave: broadcast reads
        const ulonglong2 v = kv[t];
        below += v.x < key ? 1u : 0u;
        below += v.y < key ? 1u : 0u;
      }
      s_below[part][ks] = below;
      __syncthreads();
      if (sym_thread && f) {
        const uint32_t rank = s_below[0][tid] + s_below[1][tid] + s_below[2][tid] + s_below[3][tid] - (256u - present);
        s_leaf_sym[rank] = tid;
        s_lw[rank] = (uint32_t)f;
      }
    }
    if (tid == 0) s_n = present;
  }
  __syncthreads();
  const uint32_t n = s_n;
  const uint32_t nodes = n ? 2 * n - 1 : 0, root = nodes - 1;
  if (n >= 2 && tid < 64) {
    // The merge, batched on wave 0. Let Q be the remaining nodes in the serial
    // algorithm's pick order: the merge of the leaf queue and the internal queue, a
    // leaf first on a tie. If Q[2k-1] <= Q[0] + Q[1], the next k merges pair
    // (Q[0], Q[1]), (Q[2], Q[3]), ... in that order: every node they create weighs
    // at least Q[0] + Q[1], and a new node loses every tie (it goes in after all
    // nodes of equal weight). So one round takes the first 64 entries of each queue,
    // places them in Q by merge path (each lane binary-searches the other queue),
    // and makes up to 32 merges at once. Valid codes need 13-19 rounds for 256
    // symbols (vs 255 serial merges); the result is the serial tree exactly
    // (checked against mh_code_lengths on 2000 random histograms). Weights are u32:
    // a non-root weight is below the padded pixel count <= 2^32; empty queue slots
    // hold kEnd (0xFFFFFFFF).
    const uint32_t lane = tid;
    uint32_t li = 0, ii = 0, ni = 0, m = 0;
    while (m + 1 < n) {
      // Q[0..63] by a bitonic merge in registers: key = weight : type : queue
      // position (a leaf sorts before an internal node of equal weight; each queue
      // keeps its order). min(A[i], B[63 - i]) holds the 64 smallest of both heads as
      // a bitonic sequence; six half-cleaner stages (partners from permlane32_swap,
      // ds_swizzle and DPP -- no LDS round trip) sort it.
      uint32_t q, qid;
      const uint32_t lv = s_lw[li + lane], iv = s_iw[ii + 63u - lane];
      const bool a = lv <= iv;  // equal weight: the leaf (type 0) first
      if (k32) {
        // weight (22 bits; an empty slot saturates above every real weight) : type : position (9 bits)
        uint32_t key = (min(a ? lv : iv, kW32End) << 10) | (a ? li + lane : (0x200u | (ii + 63u - lane)));
        bitonic_stage32<32>(lane, key);
        bitonic_stage32<16>(lane, key);
        bitonic_stage32<8>(lane, key);
        bitonic_stage32<4>(lane, key);
        bitonic_stage32<2>(lane, key);
        bitonic_stage32<1>(lane, key);
        q = key >> 10;
        qid = (key & 0x200u) ? n + (key & 0x1FFu) : (key & 0x1FFu);
      } else {
        uint64_t key = ((uint64_t)(a ? lv : iv) << 32) | (a ? li + lane : (0x10000u | (ii + 63u - lane)));
        bitonic_stage<32>(lane, key);
        bitonic_stage<16>(lane, key);
        bitonic_stage<8>(lane, key);
        bitonic_stage<4>(lane, key);
        bitonic_stage<2>(lane, key);
        bitonic_stage<1>(lane, key);
        q = (uint32_t)(key >> 32);
        const uint32_t kl = (uint32_t)key;
        qid = (kl & 0x10000u) ? n + (kl & 0xFFFFu) : kl;
      }
      const uint32_t s0 = __builtin_amdgcn_readlane(q, 0) + __builtin_amdgcn_readlane(q, 1);
      // ballots of plain compares, masked on the scalar side (a ballot of a combined
      // condition re-materialises it in a VGPR first)
      uint32_t k = (uint32_t)__popcll(__ballot(q <= s0) & 0xAAAAAAAAAAAAAAAAull);  // odd lanes; Q sorted: a prefix
      k = min(k, n - 1 - m);
      const uint64_t first2k = 2 * k >= 64 ? ~0ull : (1ull << (2 * k)) - 1ull;
      const uint32_t nl = (uint32_t)__popcll(__ballot(qid < n) & first2k);
      // pair j = lanes (2j, 2j+1): the odd lane adds its even neighbour (DPP) and
      // appends the new node; both lanes point their node at it
      const uint32_t qe = xor_partner<1>(lane, q);
      if (lane < 2 * k) {
        if (lane & 1u) s_iw[ni + (lane >> 1)] = qe + q;
        s_par[0][qid] = n + ni + (lane >> 1);
      }
      __builtin_amdgcn_wave_barrier();
      li += nl;
      ii += 2 * k - nl;
      ni += k;
      m += k;
    }
  }
  __syncthreads();
  // depths by pointer jumping: dep = 1 + dep(parent) over parent links, root 0
  for (uint32_t i = tid; i < nodes; i += kTreeThreads) {
    s_dep[0][i] = i == root ? 0u : 1u;
    if (i == root) s_par[0][i] = root;
  }
  __syncthreads();
  // 4 rounds: a node within 16 hops of the root gets its exact depth and the root as
  // its ancestor; any other is deeper than 16 (MH_ERR_CODE_TOO_LONG)
  uint32_t cur = 0;
  for (uint32_t step = 0; step < 4; ++step) {
    for (uint32_t i = tid; i < nodes; i += kTreeThreads) {
      const uint32_t p = s_par[cur][i];
      s_dep[cur ^ 1][i] = s_dep[cur][i] + s_dep[cur][p];
      s_par[cur ^ 1][i] = s_par[cur][p];
    }
    cur ^= 1;
    __syncthreads();
  }
  // the rest needs one thread per symbol: the other 12 waves end here (a finished
  // wave no longer counts at the workgroup barriers below)
  if (!sym_thread) return 0u;
  if (n == 0) {
    if (tid == 0) s_bad = (uint32_t)-MH_ERR_EMPTY;
  } else if (n == 1) {  // single symbol -> 1-bit code "0" (HuffmanEncoder.cpp:118-121)
    if (tid == 0) s_len[s_leaf_sym[0]] = 1;
  } else if (tid < n) {
    const uint32_t d = s_par[cur][tid] == root ? s_dep[cur][tid] : 17u;
    if (d > 16) s_bad = (uint32_t)-MH_ERR_CODE_TOO_LONG;
    s_len[s_leaf_sym[tid]] = d;
  }
  __syncthreads();
  const uint32_t L = sym_thread ? s_len[tid] : 0u;  // 0 matches no length below
  if (sym_thread) canon_out[tid] = (uint8_t)L;
  // codes per length and each symbol's rank among equal lengths (symbol order):
  // one ballot per length per wave, per-wave counts through LDS
  const uint32_t wave = tid >> 6, lane = tid & 63u;
  const uint64_t below = (1ull << lane) - 1ull;
  uint32_t in_wave = 0;
  for (uint32_t l = 1; l <= 16; ++l) {
    const uint64_t m = __ballot(L == l);
    if (L == l) in_wave = (uint32_t)__popcll(m & below);
    if (lane == 0 && wave < 4u) s_wcnt[wave][l] = (uint32_t)__popcll(m);
  }
  uint64_t bits = f * L;  // sum of count x length: wave reduction, one LDS atomic per wave
  for (int o = 32; o; o >>= 1) bits += __shfl_xor(bits, o);
  if (lane == 0 && wave < 4u) atomicAdd(&s_total, (unsigned long long)bits);
  __syncthreads();
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
  }
  __syncthreads();
  uint32_t e = 0;
  if (L && L <= 16) {
    uint32_t rank = in_wave;  // symbols of the same length before this one
    for (uint32_t w = 0; w < wave; ++w) rank += s_wcnt[w][L];
    e = ((((s_first[L] + rank) << (16 - L)) & 0xFFFFu) << 16) | L;
  }
  if constexpr (!kFused) table[tid] = e;
  __shared__ uint32_t s_bad2;
  __shared__ unsigned long long s_len_bytes;
  if (tid == 0) {
    const uint64_t total = s_total;
    const uint64_t len = (total + 7) / 8 + MH_CODES_PAD;  // + encoder's 2 and renderer's 2 zero bytes
    uint32_t bad = s_bad;
    if (!bad && (total >= (1ull << 32) || ((len + 3) & ~3ull) > codes_cap)) bad = (uint32_t)-MH_ERR_CAPACITY;
    s_bad2 = bad;
    s_len_bytes = len;
  }
  if constexpr (kFused) {
    // Publication first (the packing workgroups wait on it; nothing they read comes
    // from the bookkeeping below): each table word carries this call's tag (bits 8-15)
    // and, for a rejected frame, the bad bit (7): a packing workgroup polls the words
    // themselves, each valid on its own -- one relaxed agent-scope atomic per word, no
    // flag to order against the table (no release/acquire pair, no vmcnt reliance) and
    // no second round trip for the table after the flag.
    __syncthreads();
    __hip_atomic_store(&table[tid], e | (tag << 8) | (s_bad2 ? 0x80u : 0u), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    MH_CODE_STAMP(0, 1)
  }
  if (tid == 0) {
    const uint32_t bad = s_bad2;
    const uint64_t len = s_len_bytes;
    meta[0] = bad ? 0 : len;
    meta[1] = bad ? 0 : 1;
    meta[kTotalBits] = s_total;
    if (codes_len_out) *codes_len_out = bad ? 0 : len;
    if (status) {
      if constexpr (kFused) {
        // A packing workgroup that timed out (meta[kAbort], then its MH_ERR_HIP status)
        // must not be overwritten: every access here is sequentially consistent, so
        // either this load sees the abort, or the packer's status store follows ours.
        __hip_atomic_store(status, bad ? -(int32_t)bad : MH_OK, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_AGENT);
        if (__hip_atomic_load(reinterpret_cast<const uint32_t *>(&meta[kAbort]), __ATOMIC_SEQ_CST,
                              __HIP_MEMORY_SCOPE_AGENT))
          __hip_atomic_store(status, (int32_t)MH_ERR_HIP, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        *status = bad ? -(int32_t)bad : MH_OK;
      }
    }
  }
  if constexpr (!kFused) __syncthreads();  // s_bad2 (the fused path had its barrier above)
  return e | (s_bad2 ? 0x80u : 0u);
}

__global__ void __launch_bounds__(kTreeThreads) enc_tree_kernel(uint64_t *hist, uint8_t *canon_out,
                                                       uint32_t *table, uint64_t *meta, uint64_t *codes_len_out,
                                                       uint64_t codes_cap, int32_t *status, uint64_t nsym) {
  tree_body<false>(hist, canon_out, table, meta, codes_len_out, codes_cap, status, nsym);
}

// Block offsets, one kernel: each workgroup zeroes its share of the code words the
// packing ORs into (round_up(codes_len, 4) bytes, sized on the device), sums the
// code lengths of kScanTile blocks (HuffmanUtil.cpp:1103-1128 counts bits per block
// the same way), scans them in place and records the tile total; each packing
// workgroup sums the totals of the tiles before its own (enc_pack_kernel).
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t x) {
  const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  return x;
}

// Exclusive scan over the kScanTile threads of a workgroup: wave scans, then one
// wave scans the 16 wave totals (s_w: 16 words of LDS). Returns the prefix; *total
// gets the workgroup's sum. Ends with a barrier, so s_w may be reused at once.
__device__ __forceinline__ uint32_t wg_exclusive_scan(uint32_t x, uint32_t *s_w, uint32_t *total) {
  constexpr uint32_t kWaves = kScanTile / 64;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t incl = wave_inclusive_scan(x);
  if (lane == 63) s_w[wave] = incl;
  __syncthreads();
  if (wave == 0) {
    const uint32_t v = wave_inclusive_scan(lane < kWaves ? s_w[lane] : 0u);
    if (lane < kWaves) s_w[lane] = v;
  }
  __syncthreads();
  const uint32_t base = wave ? s_w[wave - 1] : 0u;
  *total = s_w[kWaves - 1];
  __syncthreads();
  return base + incl - x;
}

__global__ void __launch_bounds__(kScanTile) enc_scan_kernel(const uint8_t *sym, const uint32_t *table,
                                                             uint64_t nb, uint32_t *bpre, uint32_t *tsum,
                                                             uint64_t *meta, uint32_t *words) {
  __shared__ uint32_t len[256];
  __shared__ uint32_t s_w[kScanTile / 64];
  const uint32_t tid = threadIdx.x;
  if (tid < 256) len[tid] = table[tid] & 0xFFu;
  const uint64_t nw = meta[1] ? (meta[0] + 3) / 4 : 0;
  for (uint64_t i = (uint64_t)blockIdx.x * kScanTile + tid; i < nw; i += (uint64_t)gridDim.x * kScanTile)
    words[i] = 0;
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * kScanTile + tid;
  uint32_t x = 0;
  if (i < nb) {
    const uint64_t *src = reinterpret_cast<const uint64_t *>(sym + i * 64);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint64_t q = src[k];
#pragma unroll
      for (int j = 0; j < 8; ++j) x += len[(q >> (8 * j)) & 0xFF];
    }
  }
  uint32_t total;
  const uint32_t pre = wg_exclusive_scan(x, s_w, &total);
  if (i < nb) bpre[i] = pre;
  // tile totals only: each packing workgroup sums the totals before its tile
  if (tid == 0) tsum[blockIdx.x] = total;
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x00010203u); }

// Level 3 + packing, staged in LDS. Eight lanes per block, eight symbols each: a
// lane's bit position is its block's offset plus the code lengths of the lanes
// before it (a shuffle scan in the 8-lane group), so the serial chain is 8 symbols,
// not 64. A workgroup's 32 blocks own one contiguous bit range; lanes pack their
// bits MSB-first into big-endian words of that range in LDS (OR-ing the first and
// last word, which neighbouring lanes may share), then the workgroup writes the
// range out with coalesced stores, OR-ing only its first and last word (shared with
// the neighbouring workgroups) into the zeroed buffer.
constexpr uint32_t kPackBlocks = 32;
constexpr uint32_t kPackWords = kPackBlocks * 64 * 16 / 32 + 2;
__global__ void __launch_bounds__(256) enc_pack_kernel(const uint8_t *sym, const uint32_t *table,
                                                       const uint32_t *blen_prefix, const uint32_t *toff,
                                                       uint64_t nb, uint32_t *offsets, uint32_t *words,
                                                       const uint64_t *meta) {
  __shared__ uint32_t tab[256];
  __shared__ uint32_t lw[kPackWords];
  __shared__ uint32_t s_start, s_end;  // bit range of this workgroup's blocks
  const uint32_t tid = threadIdx.x, part = tid & 7u;
  if (!meta[1]) return;  // a rejected frame (status) writes nothing
  tab[tid] = table[tid];
  const uint64_t b0 = (uint64_t)blockIdx.x * kPackBlocks, b = b0 + (tid >> 3);
  const bool on = b < nb;
  const uint64_t q = on ? reinterpret_cast<const uint64_t *>(sym + b * 64)[part] : 0ull;
  // this workgroup's tile offset: wave 0 sums the scan's tile totals before it
  // (<= a few hundred L2-resident words) -- no completion ticket in the scan
  __shared__ uint32_t s_toff[2];
  const uint32_t t = (uint32_t)(b0 / kScanTile);
  if (tid < 64) {
    uint32_t acc = 0;
    for (uint32_t i = tid; i < t; i += 64) acc += toff[i];
    for (uint32_t d = 32; d; d >>= 1) acc += __shfl_xor(acc, d);
    if (tid == 0) {
      s_toff[0] = acc;
      s_toff[1] = acc + toff[t];  // the next tile's offset (read only if this tile ends here)
    }
  }
  __syncthreads();
  const uint32_t o = on ? blen_prefix[b] + s_toff[0] : 0u;
  if (on && part == 0) offsets[b] = o;
  if (tid == 0) {
    const uint64_t bn = b0 + kPackBlocks;
    s_start = o;
    s_end = bn < nb ? blen_prefix[bn] + s_toff[bn / kScanTile == t ? 0 : 1] : (uint32_t)meta[kTotalBits];
  }
  __syncthreads();
  const uint32_t w0 = s_start >> 5, nwords = ((s_end + 31) >> 5) - w0;
  for (uint32_t i = tid; i < nwords; i += 256) lw[i] = 0;
  uint32_t e[8], nbits = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    e[j] = tab[(q >> (8 * j)) & 0xFF];
    nbits += e[j] & 0xFFu;
  }
  uint32_t pre = nbits;  // inclusive scan over the block's 8 lanes
#pragma unroll
  for (uint32_t d = 1; d < 8; d <<= 1) {
    const uint32_t y = __shfl_up(pre, d, 8);
    if (part >= d) pre += y;
  }
  pre -= nbits;
  __syncthreads();
  if (on) {
    const uint32_t start = o + pre - (w0 << 5);
    uint32_t widx = start >> 5, used = start & 31u, cur = 0;
    bool first = true;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t len = e[j] & 0xFFu;
      const uint32_t c = (e[j] >> 16) >> (16 - len);  // right-aligned code
      if (used + len < 32) {
        cur |= c << (32 - used - len);
        used += len;
      } else {  // the word fills up
        const uint32_t spill = used + len - 32;
        cur |= c >> spill;
        if (first) atomicOr(&lw[widx], bswap32(cur));
        else lw[widx] = bswap32(cur);
        first = false;
        ++widx;
        cur = spill ? c << (32 - spill) : 0u;
        used = spill;
      }
    }
    if (used) atomicOr(&lw[widx], bswap32(cur));  // last, partial word: the next lane may share it
  }
  __syncthreads();
  for (uint32_t i = tid; i < nwords; i += 256) {
    const uint32_t v = lw[i];
    if (i == 0 || i == nwords - 1) {
      if (v) atomicOr(&words[w0 + i], v);
    } else {
      words[w0 + i] = v;
    }
  }
}

// ---- the fused path: enc_split_kernel (tiled) + enc_code_kernel --------------------
// One launch replaces tree + scan + pack. Workgroup 0 builds the code table
// (tree_body<true>) and publishes it through meta[kFlag]; workgroup t + 1 packs tile t
// (kCodeTile blocks, eight lanes per block, eight symbols each). While the tree is
// built, a packing workgroup loads its symbols and sums the per-tile histograms of
// the tiles before it (tile_hist, from the split), so once the table is out its bit
// offset is a 256-term dot product -- count x code length -- with no exchange between
// packing workgroups: each waits only for workgroup 0, which is dispatched first, so
// the launch cannot deadlock however few workgroups are resident. A tile's first code
// word shares bits with the previous tile's last block (every block has >= 64 bits,
// a word holds 32): the workgroup computes those bits itself from that block's
// symbols and writes the word whole; a tile leaves its own partial last word to the
// next tile (the last tile writes it and the zero pad). Every code word is written
// exactly once, so the buffer needs no clearing.
constexpr uint32_t kCodeThreads = 1024;
constexpr uint32_t kCodeMinWaves = 8;  // waves per SIMD the register budget must admit
constexpr uint32_t kCodeWaves = kCodeThreads / 64;
constexpr uint32_t kCodeWords = kCodeTile * 64 * 16 / 32 + 2;  // a tile's code words, <= 16-bit codes
static_assert(kCodeThreads == 8 * kCodeTile, "eight lanes per block");

// Inclusive prefix sum over the wave by DPP (row_shr 1/2/4/8 inside each row of 16
// lanes, then row_bcast 15 / 31 carry the row totals up): no LDS round trip.
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  return x;
}

// OR the L (1..64) right-aligned bits of v, MSB-first, into the big-endian LDS words
// lw at bit pos: at most three words, each of which a neighbouring lane may share.
__device__ __forceinline__ void or_bits(uint32_t *lw, uint32_t pos, uint64_t v, uint32_t L) {
  const uint64_t a = v << (64u - L);  // left-aligned
  const uint32_t s = pos & 31u, w = pos >> 5;
  atomicOr(&lw[w], bswap32((uint32_t)(a >> (32u + s))));
  if (s + L > 32u) atomicOr(&lw[w + 1], bswap32((uint32_t)(a >> s)));
  if (s + L > 64u) atomicOr(&lw[w + 2], bswap32((uint32_t)(a << (32u - s))));
}

struct Pixels {  // the frame as the split reads it
  const uint8_t *gray;
  uint32_t W, H, bw, vec;
  bool delta, init_byte;
};

// Tile t's code words once its first bit E is known (tab = the frame's code table in
// LDS, q = this lane's eight symbols, qp = lanes 0-7 of wave 0: the previous block's
// row symbols). Block offsets out; a tile's first word shares bits with the previous
// tile's last block (every block has >= 64 bits, a word holds 32): the workgroup
// computes those bits itself from that block's symbols and writes the word whole; a
// tile leaves its own partial last word to the next tile (the last tile writes it and
// the zero pad). Every code word is written exactly once: no clearing, no atomics.

// The stores are a fixed count of unconditional buffer stores per thread (lanes with
// nothing to store use an out-of-range offset), so the compiler counts them exactly in
// vmcnt and a persistent caller's prefetch for the next tile is never drained by them.
__device__ __forceinline__ void pack_emit(uint32_t t, uint32_t ntiles, uint32_t E, const uint32_t *tab,
                                          uint64_t q, uint64_t qp, uint64_t b, bool on, uint32_t *offsets,
                                          uint64_t nb, uint32_t *words, uint64_t words_bytes) {
  __shared__ uint32_t lw[kCodeWords];
  __shared__ uint32_t s_scan[kCodeWaves];
  const uint32_t tid = threadIdx.x, part = tid & 7u, lane = tid & 63u, wave = tid >> 6;
  (void)part;
  // this lane's codes, as two chunks of four (<= 64 bits each)
  uint64_t ch[2] = {0, 0};
  uint32_t cl[2] = {0, 0};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t e = tab[(uint32_t)(q >> (8 * j)) & 0xFFu];
    const uint32_t len = e & 0xFFu;
    ch[j >> 2] = (ch[j >> 2] << len) | ((e >> 16) >> (16 - len));
    cl[j >> 2] += len;
  }
  const uint32_t nbits = on ? cl[0] + cl[1] : 0u;
  // exclusive scan over the 1024 lanes (lane order = block order, eight lanes each)
  const uint32_t incl = wave_scan_dpp(nbits);
  if (lane == 63) s_scan[wave] = incl;
  lds_barrier();
  if (wave == 0) {
    const uint32_t v = wave_scan_dpp(lane < kCodeWaves ? s_scan[lane] : 0u);
    if (lane < kCodeWaves) s_scan[lane] = v;
  }
  lds_barrier();
  const uint32_t pre = (wave ? s_scan[wave - 1] : 0u) + incl - nbits;
  const uint32_t T = s_scan[kCodeWaves - 1];
  MH_CODE_STAMP(t + 1, 4)
  __builtin_amdgcn_raw_buffer_store_b32(E + pre, enc_rsrc(offsets, nb * 4u), (int)(on && part == 0 ? (uint32_t)b * 4u : kOob),
                                        0, 0);
  const uint32_t r = E & 31u, w0 = E >> 5, end = E + T;
  const uint32_t nwords = ((end + 31u) >> 5) - w0;
  for (uint32_t i = tid; i < nwords; i += kCodeThreads) lw[i] = 0;
  // the previous block's last r bits, the head of this tile's first word (lanes 0-7)
  uint32_t head = 0;
  if (r && wave == 0) {
    uint32_t lenp = 0;
    uint64_t acc = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t e = tab[(uint32_t)(qp >> (8 * j)) & 0xFFu];
      const uint32_t len = e & 0xFFu;
      // the lane's codes MSB-first; keep the last 64 bits (r <= 31 of them are used)
      acc = (acc << len) | ((e >> 16) >> (16 - len));
      lenp += len;
    }
    if (lane >= 8) lenp = 0;
    // bits of lanes after this one (in block order) = suffix sum over lanes 0-7
    const uint32_t incp = wave_scan_dpp(lenp);
    const uint32_t after = __builtin_amdgcn_readlane(incp, 7) - incp;
    // the word's first r bits are the block's last r bits; this lane's code bits end
    // `after` bits before the block's end, so its last bit is word bit 32 - r + after
    // (bits that would land before the word fall off the top)
    if (lane < 8 && after < r) head = (uint32_t)(acc << (32u - r + after));
    for (uint32_t o = 1; o < 8; o <<= 1) head |= __shfl_xor(head, o);
  }
  lds_barrier();
  if (on) {
    or_bits(lw, r + pre, ch[0], cl[0]);
    or_bits(lw, r + pre + cl[0], ch[1], cl[1]);
  }
  if (r && tid == 0) atomicOr(&lw[0], bswap32(head));
  lds_barrier();
  MH_CODE_STAMP(t + 1, 5)
  // a partial last word belongs to the next tile (it adds its own first bits); the
  // last tile writes it, then the zero pad up to the byte count rounded to words
  const bool last = t + 1 == ntiles;
  const uint32_t nout = (!last && (end & 31u)) ? nwords - 1 : nwords;
  const __amdgpu_buffer_rsrc_t rw = enc_rsrc(words, words_bytes);
  constexpr uint32_t kOut = (kCodeWords + kCodeThreads - 1) / kCodeThreads;
#pragma unroll
  for (uint32_t k = 0; k < kOut; ++k) {
    const uint32_t i = tid + k * kCodeThreads;
    __builtin_amdgcn_raw_buffer_store_b32(lw[min(i, kCodeWords - 1u)], rw, (int)(i < nout ? (w0 + i) * 4u : kOob), 0, 0);
  }
  // the last tile: the zero pad up to the byte count rounded to words (<= 3 words)
  const uint32_t nw = (uint32_t)(((uint64_t)(end + 7u) / 8u + MH_CODES_PAD + 3u) / 4u);
  const uint32_t ip = w0 + nwords + tid;
  __builtin_amdgcn_raw_buffer_store_b32(0u, rw, (int)(last && ip < nw ? ip * 4u : kOob), 0, 0);
}

__device__ __forceinline__ void pack_tile(uint32_t t, const Pixels px, const uint16_t *tile_hist,
                                          const uint32_t *table, uint64_t *meta, uint64_t nb, uint32_t ntiles,
                                          uint32_t *offsets, uint32_t *words, uint64_t codes_cap, int32_t *status) {
  __shared__ uint32_t tab[256];
  __shared__ uint32_t s_cnt[kCodeWaves][256];  // symbol counts of the tiles before this one, per wave
  __shared__ uint32_t s_dot[4];
  const uint32_t tid = threadIdx.x, part = tid & 7u, lane = tid & 63u, wave = tid >> 6;
  MH_CODE_STAMP(t + 1, 0)
  const uint64_t b0 = (uint64_t)t * kCodeTile, b = b0 + (tid >> 3);
  const bool on = b < nb;
  // this lane's 8 pixels (row `part` of its block) and (lanes 0-7, t > 0) the previous
  // block's rows, in flight while workgroup 0 builds the tree; the symbols are the
  // split's, re-derived here instead of going through a block-symbol buffer
  const uint64_t gq = block_row(px.gray, px.W, px.H, px.bw, nb, px.vec, b, part);
  const uint64_t gp = (t > 0 && tid < 8) ? block_row(px.gray, px.W, px.H, px.bw, nb, px.vec, b0 - 1, tid) : 0ull;
  {
    // counts of every symbol over tiles [0, t): 16-byte quad q (bins 8q..8q+7) of every
    // 32nd tile, eight loads in flight per lane (a late tile sums ~400 rows);
    // lanes l and l + 32 hold the same bins, the 16 waves' partials meet in LDS
    const uint32_t q4 = tid & 31u, j = tid >> 5;
    const uint32_t tlim = t;
    const uint4 *th = reinterpret_cast<const uint4 *>(tile_hist);
    uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t u0 = j; u0 < tlim; u0 += 32u * 8u) {
      uint4 v[8];
#pragma unroll
      for (uint32_t k = 0; k < 8; ++k) {
        const uint32_t u = u0 + 32u * k;
        v[k] = u < tlim ? th[(uint64_t)u * 32 + q4] : make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (uint32_t k = 0; k < 8; ++k) {
        const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          acc[2 * m] += w[m] & 0xFFFFu;
          acc[2 * m + 1] += w[m] >> 16;
        }
      }
    }
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      acc[m] += xor_partner<32>(lane, acc[m]);
      if (lane < 32) s_cnt[wave][8 * q4 + m] = acc[m];
    }
  }
  // (every lane runs both: the DPP reads its neighbour; blocks past nb have zero pixels)
  uint32_t first_unused;
  const uint64_t q = row_symbols(gq, part, px.delta, px.init_byte, &first_unused);
  const uint64_t qp = row_symbols(gp, tid & 7u, px.delta, px.init_byte, &first_unused);  // used by lanes 0-7 of wave 0
  const uint32_t f = wait_table(table, meta, tab, 64);  // tagged words: see tree_body
  MH_CODE_STAMP(t + 1, 1)
  if (f != 1u) {  // rejected frame (status set by the tree): write nothing
    if (f == 3u && tid == 0) {  // timed out: sticky, whenever the tree's own status lands
      __hip_atomic_store(reinterpret_cast<uint32_t *>(&meta[kAbort]), 1u, __ATOMIC_SEQ_CST,
                         __HIP_MEMORY_SCOPE_AGENT);
      if (status) __hip_atomic_store(status, (int32_t)MH_ERR_HIP, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  MH_CODE_STAMP(t + 1, 2)
  // E = first bit of this tile = sum over symbols of (count before the tile) x length
  if (wave < 4) {
    uint32_t c = 0;
#pragma unroll
    for (uint32_t j = 0; j < kCodeWaves; ++j) c += s_cnt[j][tid];
    const uint32_t x = wave_scan_dpp(c * (tab[tid] & 0xFFu));
    if (lane == 63) s_dot[wave] = x;
  }
  lds_barrier();
  const uint32_t E = s_dot[0] + s_dot[1] + s_dot[2] + s_dot[3];
  pack_emit(t, ntiles, E, tab, q, qp, b, on, offsets, nb, words, codes_cap);
#if MH_CODE_STAMPS
  if (tid == 0 && t + 1 < kCodeStampWgs)
    g_code_stamps[(t + 1) * 8 + 7] = ((unsigned long long)__builtin_amdgcn_s_getreg((3 << 11) | 20) << 32) |
                                     (unsigned long long)__smid();
  MH_CODE_STAMP(t + 1, 6)
  __builtin_amdgcn_s_waitcnt(0);
  MH_CODE_STAMP(t + 1, 3)
#endif
}

__global__ void __launch_bounds__(kCodeThreads, kCodeMinWaves) enc_code_kernel(uint64_t *hist, uint8_t *canon_out, uint32_t *table,
                                                                uint64_t *meta, uint64_t *codes_len_out,
                                                                uint64_t codes_cap, int32_t *status,
                                                                const Pixels px, const uint16_t *tile_hist,
                                                                uint64_t nb, uint32_t ntiles, uint32_t *offsets,
                                                                uint32_t *words) {
  static_assert(kTreeThreads == kCodeThreads, "workgroup 0 runs the tree");
  if (blockIdx.x == 0) {
    MH_CODE_STAMP(0, 0)
    tree_body<true>(hist, canon_out, table, meta, codes_len_out, codes_cap, status, nb * 64);
    MH_CODE_STAMP(0, 3)
    return;
  }
  pack_tile(blockIdx.x - 1, px, tile_hist, table, meta, nb, ntiles, offsets, words, codes_cap, status);
}

// ---- batched frames: enc_split_kernel (tiled) + enc_tree_batch_kernel + enc_pack_wave_kernel
// N independent frames of one size, each with its own histogram, tree and code table,
// in three launches whatever N (mh_encode_frames_device_async). The kernel boundaries
// order the phases, so no workgroup waits on another: the split (N x tiles workgroups)
// writes per-tile symbol counts; workgroup f of the tree kernel builds frame f's tree
// (tree_body) and then the frame's tile offsets (each tile's bits = its counts x the
// code lengths, exclusive scan); the pack kernel (one wave per tile, four tiles of one
// frame per workgroup) turns each tile into code words from its first bit. Frames no longer queue behind one
// workgroup's ~10 us tree each (the single-frame path): the N trees run side by side.
constexpr uint32_t kMetaWords = 32;  // per-frame meta slots (>= kGen + 1)
static_assert(kMetaWords >= kGen + 1, "meta slots");
constexpr uint32_t kTileBatch = 16;  // tiles per wave and chunk of the tile-offset pass

__global__ void __launch_bounds__(kTreeThreads) enc_tree_batch_kernel(
    uint64_t *hist, uint8_t *canon, uint32_t *table, uint64_t *meta, uint64_t *codes_len, uint64_t codes_cap,
    int32_t *status, uint64_t nb, const uint16_t *tile_hist, uint32_t ncode, uint32_t *tile_off,
    uint64_t *frame_off, uint32_t f0, uint32_t n_frames) {
  // f0: this launch's first frame of the call (its pointers start there; frame_off is
  // the call's, indexed by call frame)
  const uint32_t f = blockIdx.x, tid = threadIdx.x;
  if (frame_off && tid == 0) {  // optional: the decoder's frame_code_offsets for fixed slots
    frame_off[f0 + f] = (uint64_t)(f0 + f) * codes_cap;
    if (f0 + f + 1 == n_frames) frame_off[n_frames] = (uint64_t)n_frames * codes_cap;
  }
  // the frame's symbol counts: the sum of its tile counts (wave w: tiles w, w + 16, ...,
  // 24 8-byte loads in flight per lane, lane l: symbols 4l..4l+3), no global atomics
  __shared__ uint32_t s_part[kCodeWaves][256], s_cnt[256];
  {
    const uint32_t lane = tid & 63u, wave = tid >> 6;
    const uint2 *th = reinterpret_cast<const uint2 *>(tile_hist + (uint64_t)f * ncode * 256);
    uint32_t acc[4] = {0, 0, 0, 0};
    // 24 tiles per wave in flight (a 2048x1536 frame's 384 tiles in one round trip),
    // unconditional buffer loads (tiles past the frame read zero)
    constexpr uint32_t kDepth = 24;
    const __amdgpu_buffer_rsrc_t rth = enc_rsrc(th, (uint64_t)ncode * 512u);
    for (uint32_t t0 = wave; t0 < ncode; t0 += kCodeWaves * kDepth) {
      uint2 v[kDepth];
#pragma unroll
      for (uint32_t k = 0; k < kDepth; ++k) {
        const uint32_t t = t0 + kCodeWaves * k;
        typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));
        const v2u32 x = __builtin_amdgcn_raw_buffer_load_b64(rth, (int)(t < ncode ? t * 512u + lane * 8u : kOob), 0, 0);
        v[k] = make_uint2(x.x, x.y);
      }
#pragma unroll
      for (uint32_t k = 0; k < kDepth; ++k) {
        acc[0] += v[k].x & 0xFFFFu;
        acc[1] += v[k].x >> 16;
        acc[2] += v[k].y & 0xFFFFu;
        acc[3] += v[k].y >> 16;
      }
    }
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) s_part[wave][4 * lane + j] = acc[j];
    lds_barrier();
    if (tid < 256) {
      uint32_t c = 0;
#pragma unroll
      for (uint32_t w = 0; w < kCodeWaves; ++w) c += s_part[w][tid];
      s_cnt[tid] = c;
    }
    lds_barrier();
  }
  const uint32_t e = tree_body<false>(nullptr, canon + (uint64_t)f * 256, table + (uint64_t)f * 256,
                                      meta + (uint64_t)f * kMetaWords, codes_len ? codes_len + f : nullptr,
                                      codes_cap, status ? status + f : nullptr, nb * 64, s_cnt);
  if (tid >= 256) return;  // tree_body leaves the 256 symbol threads (4 waves)
  __shared__ uint32_t s_len[256], s_chunk[4 * kTileBatch];
  static_assert(4 * kTileBatch == 64, "one chunk total per lane of wave 0");
  s_len[tid] = e & 0x1Fu;
  lds_barrier();
  if (e & 0x80u) return;  // rejected frame (uniform): the pack kernel writes nothing
  // Tile offsets: wave w reduces tiles c + w * kTileBatch + [0, kTileBatch) of each chunk
  // of 4 * kTileBatch = 64 tiles (lane l: symbols 4l..4l+3 of a tile, one 8-byte load),
  // the next chunk's loads in flight while one is reduced; wave 0 scans the chunk's
  // totals (one per lane) with a running carry. Loads and stores are unconditional
  // buffer operations (out of range past the frame), so vmcnt counts them exactly.
  const uint32_t lane = tid & 63u, wave = tid >> 6;
  const __amdgpu_buffer_rsrc_t rth = enc_rsrc(tile_hist + (uint64_t)f * ncode * 256, (uint64_t)ncode * 512u);
  uint32_t *to = tile_off + (uint64_t)f * (ncode + 1);
  const __amdgpu_buffer_rsrc_t rto = enc_rsrc(to, (uint64_t)(ncode + 1) * 4u);
  const uint32_t l0 = s_len[4 * lane], l1 = s_len[4 * lane + 1], l2 = s_len[4 * lane + 2], l3 = s_len[4 * lane + 3];
  typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));
  const auto load_chunk = [&](uint32_t c, v2u32 (&v)[kTileBatch]) {
    const uint32_t t0 = c + wave * kTileBatch;
#pragma unroll
    for (uint32_t k = 0; k < kTileBatch; ++k)
      v[k] = __builtin_amdgcn_raw_buffer_load_b64(rth, (int)(t0 + k < ncode ? (t0 + k) * 512u + lane * 8u : kOob), 0, 0);
  };
  uint32_t carry = 0;
  v2u32 v[kTileBatch];
  load_chunk(0, v);
  for (uint32_t c = 0; c < ncode; c += 4 * kTileBatch) {
    v2u32 nv[kTileBatch];
    load_chunk(c + 4 * kTileBatch, nv);  // past the frame: all out of range
#pragma unroll
    for (uint32_t k = 0; k < kTileBatch; ++k) {
      // counts < 2^15, lengths < 2^5: 24-bit multiplies (full rate; v_mul_lo_u32 is quarter rate)
      uint32_t x = __umul24(v[k].x & 0xFFFFu, l0) + __umul24(v[k].x >> 16, l1) + __umul24(v[k].y & 0xFFFFu, l2) +
                   __umul24(v[k].y >> 16, l3);
      x = wave_scan_dpp(x);
      if (lane == 63) s_chunk[wave * kTileBatch + k] = x;  // the tile's bits (< 2^21)
    }
    lds_barrier();
    if (wave == 0) {  // 4 * kTileBatch = 64 totals: one per lane
      const uint32_t a = s_chunk[lane];
      const uint32_t incl = wave_scan_dpp(a);
      __builtin_amdgcn_raw_buffer_store_b32(carry + incl - a, rto, (int)(c + lane < ncode ? (c + lane) * 4u : kOob), 0, 0);
      carry += __builtin_amdgcn_readlane(incl, 63);
    }
    lds_barrier();
#pragma unroll
    for (uint32_t k = 0; k < kTileBatch; ++k) v[k] = nv[k];
  }
  if (tid == 0) to[ncode] = carry;
}

// Wave packing: each wave packs one tile alone, sixteen blocks per step (64 lanes: lane
// 8 m + r holds row r of the step's blocks 2 m and 2 m + 1, one 16-byte load when the
// pair shares a block row), carrying its bit position from step to step in a register
// and the step's last partial word in LDS: no workgroup barrier anywhere (a 1,024-thread
// packer that shared a tile between 16 waves spent its time in the four workgroup
// barriers per tile, profiles/r04_v4_encoder_batch_ab.txt). The next step's rows are in
// flight while a step is packed (a fixed count of unconditional buffer loads).
constexpr uint32_t kPackWaves = 4;     // waves per workgroup (independent of each other)
static_assert(kPackWaves * 64 >= 256, "one table word per thread");
constexpr uint32_t kStepBlocks = 16;
constexpr uint32_t kStepSlots = 528;   // LDS words per wave (132 quads): a step's <= 513 words + or_bits' reach
static_assert(kStepSlots >= kStepBlocks * 64 * 16 / 32 + 4 && kStepSlots % 4 == 0 && kStepSlots / 4 - 128 <= 64,
              "a step's bits (<= 16-bit codes), the carry word and or_bits' reach");

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// kPair: 8-byte aligned rows and an even frame width in blocks (a pair never straddles
// a block row): one 16-byte load per lane and step
template <bool kVec, bool kPair>
__global__ void __launch_bounds__(kPackWaves * 64) enc_pack_wave_kernel(
    const Pixels px, uint64_t gray_stride, uint64_t nb, uint32_t ncode, const uint32_t *table, const uint64_t *meta,
    const uint32_t *tile_off, uint32_t *offsets, uint8_t *codes, uint64_t codes_stride, uint32_t ncode_wg,
    const uint64_t *tile_tail) {
  // ncode_wg: workgroups per frame (ncode rounded up to kPackWaves tiles): a workgroup's
  // waves pack tiles of ONE frame and share its table, at a fixed LDS address (the
  // gathers need no per-wave base: one VALU per symbol for the address)
  __shared__ uint32_t tab[256];
  __shared__ __attribute__((aligned(16))) uint32_t s_w[kPackWaves][kStepSlots];
  // the wave index as a provably uniform value (readfirstlane): the tile, its offsets and
  // the step cursor then live in SGPRs (SALU) instead of being carried per lane
  const uint32_t lane = threadIdx.x & 63u, k = lane >> 3, r = lane & 7u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t f = blockIdx.x / ncode_wg, t = (blockIdx.x - f * ncode_wg) * kPackWaves + wave;
  if (!(uint32_t)meta[(uint64_t)f * kMetaWords + 1]) return;  // rejected frame (workgroup-uniform): nothing written
  {
    // the frame's table as len << 16 | right-aligned code (the tree's words hold the
    // code left-aligned in 16 bits): two symbols' codes combine in one v_lshl_or
    const uint32_t e = table[(uint64_t)f * 256 + threadIdx.x];
    const uint32_t L = e & 0x1Fu;
    tab[threadIdx.x] = L ? (L << 16) | ((e >> 16) >> (16u - L)) : 0u;
  }
  lds_barrier();
  if (t >= ncode) return;  // wave-uniform padding past the frame's last tile; no barrier follows
  uint32_t *lw = s_w[wave];
  const uint32_t E = tile_off[(uint64_t)f * (ncode + 1) + t];
  const uint8_t *gray = px.gray + f * gray_stride;
  const uint64_t b0 = (uint64_t)t * kBatchTile;
  const uint32_t nsteps = (uint32_t)((min<uint64_t>(kBatchTile, nb - b0) + kStepBlocks - 1) / kStepBlocks);
  const uint32_t by0 = (uint32_t)(b0 / px.bw), bx0 = (uint32_t)(b0 - (uint64_t)by0 * px.bw);
  // one descriptor from the tile's first block row: 32-bit offsets for any frame
  const uint32_t yb = by0 * 8u;
  const __amdgpu_buffer_rsrc_t rg = enc_rsrc(gray + (uint64_t)yb * px.W, (uint64_t)(px.H - yb) * px.W);
  // row r of block (bx + k, by) wrapped into the frame, zero when !live or past the frame
  // (32-bit block indices, nb < 2^26; the step's row offset uniform, r * W per lane
  // once, a wrapped block adds 8 W: no per-step v_mul_lo, which is quarter rate)
  const uint32_t nb32 = (uint32_t)nb, w8 = 8u * px.W;
  const auto load_row = [&](uint32_t sbx, uint32_t sby, uint32_t sb, uint32_t kk, uint32_t rr, uint32_t rrW,
                            bool live) -> uint64_t {
    uint32_t bx = sbx + kk, dy = 0, doff = 0;
    if (px.bw >= kStepBlocks) {  // kk < kStepBlocks: one wrap at most
      const bool wrap = bx >= px.bw;
      bx = wrap ? bx - px.bw : bx;
      dy = wrap ? 8u : 0u;
      doff = wrap ? w8 : 0u;
    } else {
      const uint32_t d = bx / px.bw;
      bx -= d * px.bw;
      dy = d * 8u;
      doff = dy * px.W;
    }
    const uint32_t ys = sby * 8u - yb;  // uniform: the step's first block row in the descriptor
    const bool in = live && sb + kk < nb32 && ys + dy + rr < px.H - yb;
    const uint32_t off = ys * px.W + doff + rrW + bx * 8u;
    if constexpr (kVec) {
      typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));
      const v2u32 v = __builtin_amdgcn_raw_buffer_load_b64(rg, (int)(in ? off : kOob), 0, 0);
      return ((uint64_t)v.y << 32) | v.x;
    } else {
      uint64_t q = 0;
#pragma unroll
      for (uint32_t c = 0; c < 8; ++c)
        q |= (uint64_t)__builtin_amdgcn_raw_buffer_load_b8(rg, (int)(in && bx * 8u + c < px.W ? off + c : kOob), 0, 0)
             << (8 * c);
      return q;
    }
  };
  uint32_t first_unused;
  // the tile's first word starts with the previous block's last E % 32 bits: lanes 0-7
  // recompute that block's codes (the previous tile leaves the shared word to this one)
  // from its symbols, which the split kept for this (tile_tail: one 64-B read)
  uint32_t head = 0;
  const uint32_t r0 = E & 31u;
  if (r0) {  // wave-uniform; t > 0 here (tile 0 starts at bit 0)
    const __amdgpu_buffer_rsrc_t rt = enc_rsrc(tile_tail + ((uint64_t)f * ncode + t - 1u) * 8u, 64u);
    typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));
    const v2u32 tv = __builtin_amdgcn_raw_buffer_load_b64(rt, (int)(lane < 8 ? lane * 8u : kOob), 0, 0);
    const uint64_t qp = ((uint64_t)tv.y << 32) | tv.x;
    uint32_t lenp = 0;
    uint64_t acc = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t e = tab[(uint32_t)(qp >> (8 * j)) & 0xFFu];
      const uint32_t len = e >> 16;
      acc = (acc << len) | (e & 0xFFFFu);  // the lane's codes MSB-first, last 64 bits
      lenp += len;
    }
    if (lane >= 8) lenp = 0;
    // bits of lanes after this one in the block; the lane's last bit lands at word bit
    // 32 - r0 + after (bits before the word fall off the top)
    const uint32_t incp = wave_scan_dpp(lenp);
    const uint32_t after = __builtin_amdgcn_readlane(incp, 7) - incp;
    uint32_t h = lane < 8 && after < r0 ? (uint32_t)(acc << (32u - r0 + after)) : 0u;
    for (uint32_t o = 1; o < 8; o <<= 1) h |= __shfl_xor(h, o);
    head = __builtin_amdgcn_readfirstlane(h);
  }
  typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
  v4u32 *lq = reinterpret_cast<v4u32 *>(lw);
  // the step's words as quads: one 16-B LDS write / read and one 16-B store per lane
  const auto clear_words = [&](uint32_t first) {
    lq[lane] = v4u32{lane == 0 ? first : 0u, 0u, 0u, 0u};
    lq[64 + lane] = v4u32{0u, 0u, 0u, 0u};
    if (lane < kStepSlots / 4 - 128) lq[128 + lane] = v4u32{0u, 0u, 0u, 0u};
  };
  clear_words(bswap32(head));
  const __amdgpu_buffer_rsrc_t rw = enc_rsrc(codes + f * codes_stride, codes_stride);
  const __amdgpu_buffer_rsrc_t ro = enc_rsrc(offsets + (uint64_t)f * nb, nb * 4u);
  uint32_t pos = E;
  uint32_t sbx = bx0, sby = by0;
  uint32_t sb = (uint32_t)b0;
  uint32_t rW = r * px.W;
  asm volatile("" : "+v"(rW));  // kept as is (else folded back into (ys + r) * W per step)
  // row r of the pair (2 k, 2 k + 1) of the step starting at block (sbx, sby) = sb
  const auto load_pair = [&](uint32_t bx_, uint32_t by_, uint32_t sb_, bool live, uint64_t &qa, uint64_t &qb) {
    if constexpr (kPair) {
      uint32_t bx = bx_ + 2u * k, doff = 0, dy = 0;
      if (px.bw >= kStepBlocks) {
        const bool wrap = bx >= px.bw;
        bx = wrap ? bx - px.bw : bx;
        dy = wrap ? 8u : 0u;
        doff = wrap ? w8 : 0u;
      } else {
        const uint32_t d = bx / px.bw;
        bx -= d * px.bw;
        dy = d * 8u;
        doff = dy * px.W;
      }
      const uint32_t ys = by_ * 8u - yb;
      const bool in = live && sb_ + 2u * k < nb32 && ys + dy + r < px.H - yb;
      // both blocks are inside the frame when the first is (an even width, an even first block)
      const v4u32 v = __builtin_amdgcn_raw_buffer_load_b128(rg, (int)(in ? ys * px.W + doff + rW + bx * 8u : kOob), 0, 0);
      qa = ((uint64_t)v.y << 32) | v.x;
      qb = ((uint64_t)v.w << 32) | v.z;
    } else {
      qa = load_row(bx_, by_, sb_, 2u * k, r, rW, live);
      qb = load_row(bx_, by_, sb_, 2u * k + 1u, r, rW, live);
    }
  };
  uint64_t qa, qb;
  load_pair(sbx, sby, sb, true, qa, qb);
  for (uint32_t s = 0; s < nsteps; ++s) {
    // the next step's rows (a dead load past the tile's last step: fixed count)
    uint32_t nbx = sbx + kStepBlocks, nby = sby;
    while (nbx >= px.bw) {  // uniform; once per step at most when bw >= kStepBlocks
      nbx -= px.bw;
      ++nby;
    }
    uint64_t na, nbq;
    load_pair(nbx, nby, sb + kStepBlocks, s + 1 < nsteps, na, nbq);
    const uint32_t ba = sb + 2u * k;
    const bool on_a = ba < nb32, on_b = ba + 1u < nb32;
    // codes MSB-first: pairs of symbols in 32 bits (v_lshl_or), chunks of four in 64
    uint64_t ch[4];
    uint32_t cl[4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint64_t v = row_symbols(h ? qb : qa, r, px.delta, px.init_byte, &first_unused);
      uint32_t pc[4], pl[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t e0 = tab[(uint32_t)(v >> (16 * j)) & 0xFFu], e1 = tab[(uint32_t)(v >> (16 * j + 8)) & 0xFFu];
        const uint32_t l1 = e1 >> 16;
        pc[j] = ((e0 & 0xFFFFu) << l1) | (e1 & 0xFFFFu);
        pl[j] = (e0 >> 16) + l1;
      }
      ch[2 * h] = ((uint64_t)pc[0] << pl[1]) | pc[1];
      ch[2 * h + 1] = ((uint64_t)pc[2] << pl[3]) | pc[3];
      cl[2 * h] = pl[0] + pl[1];
      cl[2 * h + 1] = pl[2] + pl[3];
    }
    const uint32_t na_bits = on_a ? cl[0] + cl[1] : 0u, nb_bits = on_b ? cl[2] + cl[3] : 0u;
    // bit order: block 2 k (rows 0-7), then block 2 k + 1: one scan of A | B << 16 (each
    // half's sum over the wave <= 8,192), the pair's start and its A total by broadcast
    const uint32_t x = na_bits | (nb_bits << 16);
    const uint32_t S = wave_scan_dpp(x), ex = S - x;
    const uint32_t g = __shfl(ex, lane & ~7u), ge = __shfl(S, lane | 7u);
    const uint32_t Tw = __builtin_amdgcn_readlane(S, 63);
    const uint32_t T = (Tw & 0xFFFFu) + (Tw >> 16);
    const uint32_t start = (g & 0xFFFFu) + (g >> 16);             // the pair's first bit (step-relative)
    const uint32_t atot = (ge & 0xFFFFu) - (g & 0xFFFFu);         // block 2 k's bits
    const uint32_t pa = (g >> 16) + (ex & 0xFFFFu);                // this row of block 2 k
    const uint32_t pb = (g & 0xFFFFu) + atot + (ex >> 16);         // this row of block 2 k + 1
    // block offsets: lane r = 0 writes block 2 k's, lane r = 1 block 2 k + 1's
    const bool wo = r == 0 ? on_a : r == 1 ? on_b : false;
    __builtin_amdgcn_raw_buffer_store_b32(pos + start + (r == 1 ? atot : 0u), ro, (int)(wo ? (ba + r) * 4u : kOob), 0,
                                          0);
    const uint32_t rr = pos & 31u;
    if (!MH_DIAG_PACK_NO_OR && on_a) {
      or_bits(lw, rr + pa, ch[0], cl[0]);
      or_bits(lw, rr + pa + cl[0], ch[1], cl[1]);
    }
    if (!MH_DIAG_PACK_NO_OR && on_b) {
      or_bits(lw, rr + pb, ch[2], cl[2]);
      or_bits(lw, rr + pb + cl[2], ch[3], cl[3]);
    }
    wave_sync();
    // whole words out; the last partial word stays as the next step's first
    const uint32_t nfull = (rr + T) >> 5, w0 = pos >> 5, nq4 = nfull >> 2;
    const v4u32 q0 = lq[lane], q1 = lq[64 + lane];                    // words 4 lane .., 256 + 4 lane ..
    const uint32_t tail = lw[min(4u * nq4 + lane, kStepSlots - 1u)];  // lanes < nfull % 4: the last words
    const uint32_t carry = lw[nfull];
    __builtin_amdgcn_raw_buffer_store_b128(q0, rw, (int)(lane < nq4 ? (w0 + 4u * lane) * 4u : kOob), 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(q1, rw, (int)(64u + lane < nq4 ? (w0 + 256u + 4u * lane) * 4u : kOob), 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(tail, rw, (int)(lane < (nfull & 3u) ? (w0 + 4u * nq4 + lane) * 4u : kOob), 0,
                                          0);
    wave_sync();
    clear_words(carry);
    wave_sync();
    pos += T;
    qa = na;
    qb = nbq;
    sbx = nbx;
    sby = nby;
    sb += kStepBlocks;
  }
  // the last tile writes its partial last word, then the zero pad up to the byte count
  // rounded to words (the others leave that word to the next tile)
  if (t + 1 == ncode) {
    const uint32_t nw = (uint32_t)(((uint64_t)(pos + 7u) / 8u + MH_CODES_PAD + 3u) / 4u);
    const uint32_t w = (pos >> 5) + lane;
    const uint32_t val = lane == 0 ? lw[0] : 0u;
    __builtin_amdgcn_raw_buffer_store_b32(val, rw, (int)(w < nw ? w * 4u : kOob), 0, 0);
  }
}

struct BatchWorkspace {  // per-frame slices, each part 256-B aligned; nothing needs zeroing
  uint32_t *table;      // n x 256
  uint64_t *meta;       // n x kMetaWords
  uint16_t *tile_hist;  // n x ncode x 256
  uint32_t *tile_off;   // n x (ncode + 1)
  uint64_t *tile_tail;  // n x ncode x 8: the symbols of each tile's last block (rows as u64)
};

uint64_t carve_batch(uint8_t *base, uint64_t nb, uint32_t n, BatchWorkspace *w) {
  const uint64_t ncode = (nb + kBatchTile - 1) / kBatchTile;
  uint64_t o = 0;
  if (w) w->table = reinterpret_cast<uint32_t *>(base + o);
  o += align256((uint64_t)n * 256 * 4);
  if (w) w->meta = reinterpret_cast<uint64_t *>(base + o);
  o += align256((uint64_t)n * kMetaWords * 8);
  if (w) w->tile_hist = reinterpret_cast<uint16_t *>(base + o);
  o += align256((uint64_t)n * ncode * 256 * 2);
  if (w) w->tile_off = reinterpret_cast<uint32_t *>(base + o);
  o += align256((uint64_t)n * (ncode + 1) * 4);
  if (w) w->tile_tail = reinterpret_cast<uint64_t *>(base + o);
  o += align256((uint64_t)n * ncode * 64);
  return o;
}

}  // namespace

extern "C" {

// Frames of <= kFusedMaxTiles code tiles take the two-launch path by default
// (enc_split_kernel tiled, then enc_code_kernel: the tree in workgroup 0 while the
// packers sum the earlier tiles' histograms); larger frames take the four-kernel path
// (split, tree, scan, pack). MH_ENCODE_KERNELS=4 forces the four-kernel path for
// every size (A/B, tested); any other value keeps the default.
static int encode_kernels() {
  static const int k = [] {
    const char *v = std::getenv("MH_ENCODE_KERNELS");
    return v && std::strcmp(v, "4") == 0 ? 4 : 2;
  }();
  return k;
}

// mh_encode_frame_device_async's workspace; mh_encode_frame_device needs kResultBytes
// more (see mh_encode_workspace_bytes in the header: it reports the larger figure).
static size_t async_workspace_bytes(uint32_t width, uint32_t height) {
  const uint64_t nb = (uint64_t)((width + 7) / 8) * ((height + 7) / 8);
  return (size_t)carve(nullptr, nb, nullptr);
}

#if MH_CODE_STAMPS
int mh_diag_code_stamps_reset(void) {
  static unsigned long long z[kCodeStampWgs * 8];
  for (auto &v : z) v = 0;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_code_stamps), z, sizeof(z), 0, hipMemcpyHostToDevice) == hipSuccess &&
                 hipMemcpyToSymbol(HIP_SYMBOL(g_split_stamps), z, sizeof(z), 0, hipMemcpyHostToDevice) == hipSuccess
             ? 0
             : -1;
}
int mh_diag_code_stamps(unsigned long long *host, size_t n) {
  if (n > kCodeStampWgs * 8) n = kCodeStampWgs * 8;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_code_stamps), n * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? (int)n : -1;
}
int mh_diag_split_stamps(unsigned long long *host, size_t n) {
  if (n > kCodeStampWgs * 8) n = kCodeStampWgs * 8;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_split_stamps), n * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? (int)n : -1;
}
#endif

size_t mh_encode_workspace_bytes(uint32_t width, uint32_t height) {
  return async_workspace_bytes(width, height) + kResultBytes;
}

int mh_encode_frame_device_async(const uint8_t *d_gray, uint32_t width, uint32_t height, uint32_t flags,
                                 uint8_t *d_canon_header, uint8_t *d_codes, uint64_t codes_cap,
                                 uint64_t *d_codes_len, uint32_t *d_block_offsets, uint8_t *d_block_init,
                                 int32_t *d_status, void *d_workspace, size_t workspace_bytes, void *stream) {
  if (!d_gray || !d_canon_header || !d_codes || !d_block_offsets || !d_workspace)
    return MH_ERR_INVALID_ARG;
  if (flags & ~(MH_FLAG_NO_DELTA | MH_ENCODE_WORKSPACE_ZEROED)) return MH_ERR_INVALID_ARG;
  if (!width || !height || width > MH_MAX_DIM || height > MH_MAX_DIM) return MH_ERR_DIMS;
  if (((uintptr_t)d_codes & 3u) || ((uintptr_t)d_workspace & 255u)) return MH_ERR_ALIGN;
  const uint32_t bw = (width + 7) / 8, bh = (height + 7) / 8;
  const uint64_t nb = (uint64_t)bw * bh;
  if (workspace_bytes < async_workspace_bytes(width, height)) return MH_ERR_CAPACITY;
  Workspace w;
  carve(static_cast<uint8_t *>(d_workspace), nb, &w);
  hipStream_t s = (hipStream_t)stream;
  const uint32_t g256 = (uint32_t)((nb + 255) / 256);
  const uint64_t ntiles = (nb + kScanTile - 1) / kScanTile;
  if (g256 == 0 || ntiles > 0xFFFFFFFFull) return MH_ERR_CAPACITY;

  const uint64_t ncode = (nb + kCodeTile - 1) / kCodeTile;
  // Per-call state: the tree zeroes the histogram after reading it, and the fused
  // path's table words carry a call tag from meta[kGen], which the split kernel
  // advances once per call. Without MH_ENCODE_WORKSPACE_ZEROED the histogram, the code
  // table and meta[0 .. kGen) are zeroed (contiguous, one memset), meta[kGen] is NOT:
  // a zeroed (or garbage-free) table word carries tag 0, which no call uses, and the
  // tag still differs from the previous call's, so a packer can take neither the
  // previous call's table words -- even from a stale cache line -- nor a cleared one.
  // (zeroing meta[kGen] too gave every call the same tag.)
  const size_t state_bytes = align256(kHistParts * 256 * 8) + align256(256 * 4) + kGen * 8;
  if (!(flags & MH_ENCODE_WORKSPACE_ZEROED) && hipMemsetAsync(w.hist, 0, state_bytes, s) != hipSuccess)
    return MH_ERR_HIP;
  flags &= ~MH_ENCODE_WORKSPACE_ZEROED;
  const uint32_t vec = (width % 8 == 0 && ((uintptr_t)d_gray & 7u) == 0) ? 1u : 0u;
  const int path = encode_kernels();
  if (ncode <= kFusedMaxTiles && path == 2) {
    // two launches: the tiled split, then tree + offsets + packing in one kernel
    hipLaunchKernelGGL((vec ? enc_split_kernel<true, true> : enc_split_kernel<false, true>), dim3((uint32_t)ncode),
                       dim3(256), 0, s, d_gray, width, height, bw, nb, flags, nullptr, d_block_init, w.hist, w.tile_hist, w.meta, (uint32_t)ncode, 0ull,
                       nullptr);
    const Pixels px{d_gray, width, height, bw, vec, !(flags & MH_FLAG_NO_DELTA), d_block_init != nullptr};
    hipLaunchKernelGGL(enc_code_kernel, dim3((uint32_t)ncode + 1), dim3(kCodeThreads), 0, s, w.hist,
                       d_canon_header, w.table, w.meta, d_codes_len, codes_cap, d_status, px, w.tile_hist, nb,
                       (uint32_t)ncode, d_block_offsets, reinterpret_cast<uint32_t *>(d_codes));
    return hipGetLastError() == hipSuccess ? MH_OK : MH_ERR_HIP;
  }
  const uint32_t gsplit = (uint32_t)std::min<uint64_t>((nb + 31) / 32, kSplitWgs);
  hipLaunchKernelGGL((vec ? enc_split_kernel<true, false> : enc_split_kernel<false, false>), dim3(gsplit), dim3(256), 0,
                     s, d_gray, width, height, bw, nb, flags, w.sym, d_block_init, w.hist, nullptr, w.meta, 0u, 0ull, nullptr);
  hipLaunchKernelGGL(enc_tree_kernel, dim3(1), dim3(kTreeThreads), 0, s, w.hist, d_canon_header, w.table, w.meta,
                     d_codes_len, codes_cap, d_status, nb * 64);
  hipLaunchKernelGGL(enc_scan_kernel, dim3((uint32_t)ntiles), dim3(kScanTile), 0, s, w.sym, w.table, nb, w.blen,
                     w.tsum, w.meta, reinterpret_cast<uint32_t *>(d_codes));
  hipLaunchKernelGGL(enc_pack_kernel, dim3((uint32_t)((nb + kPackBlocks - 1) / kPackBlocks)), dim3(256), 0, s, w.sym, w.table, w.blen, w.tsum, nb,
                     d_block_offsets, reinterpret_cast<uint32_t *>(d_codes), w.meta);
  return hipGetLastError() == hipSuccess ? MH_OK : MH_ERR_HIP;
}

int mh_encode_frame_device(const uint8_t *d_gray, uint32_t width, uint32_t height, uint32_t flags,
                           uint8_t canon_header[256], uint8_t *d_codes, uint64_t codes_cap,
                           uint64_t *codes_len, uint32_t *d_block_offsets, uint8_t *d_block_init,
                           void *d_workspace, size_t workspace_bytes, void *stream) {
  if (!canon_header || !codes_len) return MH_ERR_INVALID_ARG;
  if (workspace_bytes < mh_encode_workspace_bytes(width, height)) return MH_ERR_CAPACITY;
  // header, byte count and status land at the end of the workspace, then come over
  // in one copy and one synchronisation
  uint8_t *res = static_cast<uint8_t *>(d_workspace) + (workspace_bytes - kResultBytes) / 256 * 256;
  int rc = mh_encode_frame_device_async(d_gray, width, height, flags, res, d_codes, codes_cap,
                                        reinterpret_cast<uint64_t *>(res + 256), d_block_offsets, d_block_init,
                                        reinterpret_cast<int32_t *>(res + 264), d_workspace,
                                        (workspace_bytes - kResultBytes) / 256 * 256, stream);
  if (rc != MH_OK) return rc;
  uint8_t host[kResultBytes];
  hipStream_t s = (hipStream_t)stream;
  if (hipMemcpyAsync(host, res, kResultBytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return MH_ERR_HIP;
  int32_t status;
  std::memcpy(&status, host + 264, 4);
  if (status != MH_OK) return status;
  std::memcpy(canon_header, host, 256);
  std::memcpy(codes_len, host + 256, 8);
  return MH_OK;
}

size_t mh_encode_frames_workspace_bytes(uint32_t width, uint32_t height, uint32_t n_frames) {
  const uint64_t nb = (uint64_t)((width + 7) / 8) * ((height + 7) / 8);
  return (size_t)carve_batch(nullptr, nb, n_frames, nullptr);
}

int mh_encode_frames_device_async(const uint8_t *d_gray, uint64_t gray_frame_stride, uint32_t n_frames,
                                  uint32_t width, uint32_t height, uint32_t flags, uint8_t *d_canon_headers,
                                  uint8_t *d_codes, uint64_t codes_frame_stride, uint64_t *d_codes_len,
                                  uint64_t *d_frame_code_offsets, uint32_t *d_block_offsets, uint8_t *d_block_init,
                                  int32_t *d_status, void *d_workspace, size_t workspace_bytes, void *stream) {
  if (!d_gray || !d_canon_headers || !d_codes || !d_block_offsets || !d_workspace || !n_frames)
    return MH_ERR_INVALID_ARG;
  if (flags & ~(MH_FLAG_NO_DELTA | MH_ENCODE_WORKSPACE_ZEROED)) return MH_ERR_INVALID_ARG;
  if (!width || !height || width > MH_MAX_DIM || height > MH_MAX_DIM) return MH_ERR_DIMS;
  if (((uintptr_t)d_codes & 15u) || (codes_frame_stride & 15u) || ((uintptr_t)d_workspace & 255u))
    return MH_ERR_ALIGN;
  if (gray_frame_stride < (uint64_t)width * height && n_frames > 1) return MH_ERR_CAPACITY;
  const uint32_t bw = (width + 7) / 8, bh = (height + 7) / 8;
  const uint64_t nb = (uint64_t)bw * bh;
  const uint64_t ncode = (nb + kBatchTile - 1) / kBatchTile;
  if (ncode * n_frames > 0x7FFFFFFFull || n_frames > 0x7FFFFFFFu) return MH_ERR_CAPACITY;
  if (workspace_bytes < mh_encode_frames_workspace_bytes(width, height, n_frames)) return MH_ERR_CAPACITY;
  BatchWorkspace w;
  carve_batch(static_cast<uint8_t *>(d_workspace), nb, n_frames, &w);
  hipStream_t s = (hipStream_t)stream;
  // every part of the workspace is written before it is read within the call (the tile
  // counts by the split, the tables and tile offsets by the trees): nothing to clear
  flags &= ~MH_ENCODE_WORKSPACE_ZEROED;
  const uint32_t vec = (width % 8 == 0 && ((uintptr_t)d_gray & 7u) == 0 && (gray_frame_stride & 7u) == 0) ? 1u : 0u;
  const Pixels px0{d_gray, width, height, bw, vec, !(flags & MH_FLAG_NO_DELTA), d_block_init != nullptr};
  // frames [f0, f0 + m): split, trees, packing on stream st
  const auto sub_batch = [&](hipStream_t st, uint32_t f0, uint32_t m) {
    const uint32_t nt = (uint32_t)(ncode * m);
    const uint8_t *gray = d_gray + f0 * gray_frame_stride;
    uint8_t *binit = d_block_init ? d_block_init + (uint64_t)f0 * nb : nullptr;
    uint16_t *th = w.tile_hist + (uint64_t)f0 * ncode * 256;
    uint32_t *table = w.table + (uint64_t)f0 * 256;
    uint64_t *meta = w.meta + (uint64_t)f0 * kMetaWords;
    uint32_t *to = w.tile_off + (uint64_t)f0 * (ncode + 1);
    // one workgroup per tile (a persistent split with the next tile's rows in flight
    // measured slower: profiles/r04_v4_encoder_batch_ab.txt)
    uint64_t *tail = w.tile_tail + (uint64_t)f0 * ncode * 8;
    hipLaunchKernelGGL((vec ? enc_split_kernel<true, true, kBatchTile> : enc_split_kernel<false, true, kBatchTile>), dim3(nt),
                       dim3(256), 0, st,
                       gray, width, height, bw, nb, flags, nullptr, binit, nullptr, th, nullptr, (uint32_t)ncode,
                       gray_frame_stride, tail);
    hipLaunchKernelGGL(enc_tree_batch_kernel, dim3(m), dim3(kTreeThreads), 0, st, nullptr,
                       d_canon_headers + (uint64_t)f0 * 256, table, meta, d_codes_len ? d_codes_len + f0 : nullptr,
                       codes_frame_stride, d_status ? d_status + f0 : nullptr, nb, th, (uint32_t)ncode, to,
                       d_frame_code_offsets, f0, n_frames);
    Pixels px = px0;
    px.gray = gray;
    const uint32_t ncode_wg = (uint32_t)((ncode + kPackWaves - 1) / kPackWaves);
    hipLaunchKernelGGL((!vec ? enc_pack_wave_kernel<false, false>
                            : bw % 2 ? enc_pack_wave_kernel<true, false> : enc_pack_wave_kernel<true, true>),
                       dim3(ncode_wg * m), dim3(kPackWaves * 64), 0, st, px, gray_frame_stride, nb, (uint32_t)ncode, table,
                       meta, to, d_block_offsets + (uint64_t)f0 * nb, d_codes + f0 * codes_frame_stride,
                       codes_frame_stride, ncode_wg, tail);
  };
  // One sub-batch: splitting the call into sub-batches alternated over a second stream
  // (trees beside another sub-batch's split / packing) measured slower, and the packer's
  // pixel re-reads did not drop (profiles/r04_v4_encoder_batch_ab.txt).
  sub_batch(s, 0, n_frames);
  return hipGetLastError() == hipSuccess ? MH_OK : MH_ERR_HIP;
}

}  // extern "C"

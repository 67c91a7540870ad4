// mh_encode.hip -- GPU encoder for 8-bit grayscale frames:
// the producer side of the path, byte-identical to mh_encode_frame (mh_host.cpp),
// which itself reproduces the reference encoder:
//   split + deltas   Shared/Util.m:233-323, Shared/AAPLRenderer.m:432-515 (one thread
//                    per 8x8 block, zero padding past W/H, optional init byte :449-473)
//   histogram        HuffmanEncoder.cpp:310-330 (symbol counts; LDS then global atomics)
//   code lengths     HuffmanEncoder.cpp:29-145 -- on the HOST from the 256 counts (the
//                    reference's node-array tie-breaking is inherently sequential and
//                    tiny), mh_code_lengths + canonical codes huff_util.hpp:94-193
//   block offsets    HuffmanUtil.cpp:1103-1128 -- an exclusive prefix sum of the
//                    per-block code-length sums
//   bit packing      HuffmanEncoder.cpp:211-381 -- MSB-first; each block writes its own
//                    words, OR-ing the two it may share with its neighbours
// The call synchronises its stream once (the 1 KB histogram comes to the host).
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <cstring>

#include "../../include/metalhuffman.h"

extern "C" int mh_code_lengths(const uint64_t freq[256], uint8_t canon_header[256]);
extern "C" int mh_canonical_codes(const uint8_t canon_header[256], uint16_t codes[256]);

namespace {

constexpr uint32_t kScanTile = 1024;  // blocks per workgroup in the offsets scan

struct Workspace {  // carved out of the caller's workspace, 256-B aligned parts
  uint8_t *sym;       // nb * 64 block symbols
  uint32_t *blen;     // nb per-block bit lengths
  uint32_t *tsum;     // ceil(nb / kScanTile) tile sums (then tile offsets)
  uint64_t *hist;     // 256 counts
  uint32_t *table;    // 256 x (code_lj16 << 16 | len)
};

constexpr uint64_t align256(uint64_t x) { return (x + 255) & ~255ull; }

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
  o += align256(256 * 8);
  if (w) w->table = reinterpret_cast<uint32_t *>(base + o);
  o += align256(256 * 4);
  return o;
}

// One thread per block: pixels -> 64 symbols (block order, row-major inside the
// block, zero past the frame edge), per-block deltas, histogram.
__global__ void __launch_bounds__(256) enc_split_kernel(const uint8_t *gray, uint32_t W, uint32_t H,
                                                        uint32_t bw, uint64_t nb, uint32_t flags,
                                                        uint8_t *sym, uint8_t *block_init,
                                                        uint64_t *hist) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b < nb) {
    const uint32_t bx = (uint32_t)(b % bw), by = (uint32_t)(b / bw);
    uint8_t v[64];
    for (uint32_t r = 0; r < 8; ++r) {
      const uint32_t y = by * 8 + r;
      for (uint32_t c = 0; c < 8; ++c) {
        const uint32_t x = bx * 8 + c;
        v[r * 8 + c] = (y < H && x < W) ? gray[(uint64_t)y * W + x] : 0;
      }
    }
    if (!(flags & MH_FLAG_NO_DELTA)) {
      uint8_t prev = 0;
      for (int i = 0; i < 64; ++i) {
        const uint8_t cur = v[i];
        v[i] = (uint8_t)(cur - prev);
        prev = cur;
      }
      if (block_init) {
        block_init[b] = v[0];
        v[0] = 0;
      }
    } else if (block_init) {
      block_init[b] = 0;
    }
    uint64_t *dst = reinterpret_cast<uint64_t *>(sym + b * 64);
    for (int k = 0; k < 8; ++k) {
      uint64_t q = 0;
      for (int j = 0; j < 8; ++j) q |= (uint64_t)v[k * 8 + j] << (8 * j);
      dst[k] = q;
    }
    for (int i = 0; i < 64; ++i) atomicAdd(&h[v[i]], 1u);
  }
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd((unsigned long long *)&hist[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

// Per-block code-length sums.
__global__ void __launch_bounds__(256) enc_blen_kernel(const uint8_t *sym, const uint32_t *table,
                                                       uint64_t nb, uint32_t *blen) {
  __shared__ uint32_t len[256];
  len[threadIdx.x] = table[threadIdx.x] & 0xFFu;
  __syncthreads();
  const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  const uint64_t *src = reinterpret_cast<const uint64_t *>(sym + b * 64);
  uint32_t n = 0;
  for (int k = 0; k < 8; ++k) {
    const uint64_t q = src[k];
    for (int j = 0; j < 8; ++j) n += len[(q >> (8 * j)) & 0xFF];
  }
  blen[b] = n;
}

// Exclusive scan, level 1: each workgroup scans kScanTile block lengths in place
// and records the tile total.
__global__ void __launch_bounds__(kScanTile) enc_scan_tiles(uint32_t *blen, uint64_t nb, uint32_t *tsum) {
  __shared__ uint32_t s[kScanTile];
  const uint64_t i = (uint64_t)blockIdx.x * kScanTile + threadIdx.x;
  const uint32_t x = i < nb ? blen[i] : 0u;
  s[threadIdx.x] = x;
  __syncthreads();
  for (uint32_t d = 1; d < kScanTile; d <<= 1) {  // Hillis-Steele inclusive scan
    const uint32_t add = threadIdx.x >= d ? s[threadIdx.x - d] : 0u;
    __syncthreads();
    s[threadIdx.x] += add;
    __syncthreads();
  }
  if (i < nb) blen[i] = s[threadIdx.x] - x;
  if (threadIdx.x == kScanTile - 1) tsum[blockIdx.x] = s[threadIdx.x];
}

// Level 2: one workgroup turns the tile totals into tile offsets (serial chunks).
__global__ void __launch_bounds__(kScanTile) enc_scan_totals(uint32_t *tsum, uint64_t ntiles) {
  __shared__ uint32_t s[kScanTile];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint64_t base = 0; base < ntiles; base += kScanTile) {
    const uint64_t i = base + threadIdx.x;
    const uint32_t x = i < ntiles ? tsum[i] : 0u;
    s[threadIdx.x] = x;
    __syncthreads();
    for (uint32_t d = 1; d < kScanTile; d <<= 1) {
      const uint32_t add = threadIdx.x >= d ? s[threadIdx.x - d] : 0u;
      __syncthreads();
      s[threadIdx.x] += add;
      __syncthreads();
    }
    if (i < ntiles) tsum[i] = carry + s[threadIdx.x] - x;
    __syncthreads();
    if (threadIdx.x == kScanTile - 1) carry += s[threadIdx.x];
    __syncthreads();
  }
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x00010203u); }

// Level 3 + packing: block b's offset = its in-tile prefix + its tile's offset;
// the block's 64 codes go out MSB-first as big-endian words. Interior words are
// the block's alone (plain stores); its first and last word may be shared with
// the neighbouring blocks (atomic OR into the zeroed buffer).
__global__ void __launch_bounds__(256) enc_pack_kernel(const uint8_t *sym, const uint32_t *table,
                                                       const uint32_t *blen_prefix, const uint32_t *toff,
                                                       uint64_t nb, uint32_t *offsets, uint32_t *words) {
  __shared__ uint32_t tab[256];
  tab[threadIdx.x] = table[threadIdx.x];
  __syncthreads();
  const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  const uint32_t o = blen_prefix[b] + toff[b / kScanTile];
  offsets[b] = o;
  const uint64_t *src = reinterpret_cast<const uint64_t *>(sym + b * 64);
  uint32_t widx = o >> 5, used = o & 31u, cur = 0;
  bool first = true;
  auto emit = [&](bool shared) {
    if (shared) atomicOr(&words[widx], bswap32(cur));
    else words[widx] = bswap32(cur);
  };
  for (int k = 0; k < 8; ++k) {
    const uint64_t q = src[k];
    for (int j = 0; j < 8; ++j) {
      const uint32_t e = tab[(q >> (8 * j)) & 0xFF];
      const uint32_t len = e & 0xFFu;
      const uint32_t c = (e >> 16) >> (16 - len);  // right-aligned code
      if (used + len < 32) {
        cur |= c << (32 - used - len);
        used += len;
      } else {  // the word fills up
        const uint32_t spill = used + len - 32;
        cur |= c >> spill;
        emit(first);
        first = false;
        ++widx;
        cur = spill ? c << (32 - spill) : 0u;
        used = spill;
      }
    }
  }
  if (used) emit(true);  // last, partial word: the next block may share it
}

}  // namespace

extern "C" {

size_t mh_encode_workspace_bytes(uint32_t width, uint32_t height) {
  const uint64_t nb = (uint64_t)((width + 7) / 8) * ((height + 7) / 8);
  return (size_t)carve(nullptr, nb, nullptr);
}

int mh_encode_frame_device(const uint8_t *d_gray, uint32_t width, uint32_t height, uint32_t flags,
                           uint8_t canon_header[256], uint8_t *d_codes, uint64_t codes_cap,
                           uint64_t *codes_len, uint32_t *d_block_offsets, uint8_t *d_block_init,
                           void *d_workspace, size_t workspace_bytes, void *stream) {
  if (!d_gray || !canon_header || !d_codes || !codes_len || !d_block_offsets || !d_workspace)
    return MH_ERR_INVALID_ARG;
  if (flags & ~MH_FLAG_NO_DELTA) return MH_ERR_INVALID_ARG;
  if (!width || !height || width > MH_MAX_DIM || height > MH_MAX_DIM) return MH_ERR_DIMS;
  if (((uintptr_t)d_codes & 3u) || ((uintptr_t)d_workspace & 255u)) return MH_ERR_ALIGN;
  const uint32_t bw = (width + 7) / 8, bh = (height + 7) / 8;
  const uint64_t nb = (uint64_t)bw * bh;
  if (workspace_bytes < mh_encode_workspace_bytes(width, height)) return MH_ERR_CAPACITY;
  Workspace w;
  carve(static_cast<uint8_t *>(d_workspace), nb, &w);
  hipStream_t s = (hipStream_t)stream;
  const uint32_t g256 = (uint32_t)((nb + 255) / 256);
  const uint64_t ntiles = (nb + kScanTile - 1) / kScanTile;
  if (g256 == 0 || ntiles > 0xFFFFFFFFull) return MH_ERR_CAPACITY;

  if (hipMemsetAsync(w.hist, 0, 256 * 8, s) != hipSuccess) return MH_ERR_HIP;
  hipLaunchKernelGGL(enc_split_kernel, dim3(g256), dim3(256), 0, s, d_gray, width, height, bw, nb, flags,
                     w.sym, d_block_init, w.hist);
  uint64_t hist[256];
  if (hipGetLastError() != hipSuccess ||
      hipMemcpyAsync(hist, w.hist, sizeof(hist), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return MH_ERR_HIP;

  // host: the reference's tree on 256 counts, canonical codes, sizes
  int rc = mh_code_lengths(hist, canon_header);
  if (rc != MH_OK) return rc;
  uint16_t cc[256];
  rc = mh_canonical_codes(canon_header, cc);
  if (rc != MH_OK) return rc;
  uint64_t total_bits = 0;
  uint32_t table[256];
  for (int i = 0; i < 256; ++i) {
    total_bits += hist[i] * canon_header[i];
    table[i] = ((uint32_t)cc[i] << 16) | canon_header[i];
  }
  if (total_bits >= (1ull << 32)) return MH_ERR_CAPACITY;  // u32 block offsets
  const uint64_t payload = (total_bits + 7) / 8;
  const uint64_t len = payload + MH_CODES_PAD;  // + encoder's 2 and renderer's 2 zero bytes
  const uint64_t zero_bytes = (len + 3) & ~3ull;
  if (zero_bytes > codes_cap) return MH_ERR_CAPACITY;

  if (hipMemcpyAsync(w.table, table, sizeof(table), hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemsetAsync(d_codes, 0, zero_bytes, s) != hipSuccess)
    return MH_ERR_HIP;
  hipLaunchKernelGGL(enc_blen_kernel, dim3(g256), dim3(256), 0, s, w.sym, w.table, nb, w.blen);
  hipLaunchKernelGGL(enc_scan_tiles, dim3((uint32_t)ntiles), dim3(kScanTile), 0, s, w.blen, nb, w.tsum);
  hipLaunchKernelGGL(enc_scan_totals, dim3(1), dim3(kScanTile), 0, s, w.tsum, ntiles);
  hipLaunchKernelGGL(enc_pack_kernel, dim3(g256), dim3(256), 0, s, w.sym, w.table, w.blen, w.tsum, nb,
                     d_block_offsets, reinterpret_cast<uint32_t *>(d_codes));
  if (hipGetLastError() != hipSuccess) return MH_ERR_HIP;
  *codes_len = len;
  return MH_OK;
}

}  // extern "C"

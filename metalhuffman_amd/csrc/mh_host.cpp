// mh_host.cpp -- host-side producer of the MI355X Huffman block codec.
//
// Clean-room C++ re-derivation of the reference's CPU codec so that the frames
// the GPU decoder consumes are byte-identical to what mdejong/MetalHuffman's
// encoder emits:
//   * block split            Shared/Util.m:233-323
//   * per-block byte deltas  Shared/HuffmanUtil.cpp:21-85, :1133-1145
//   * Huffman code lengths   Shared/HuffmanEncoder.cpp:29-145 (node-array tie-breaking)
//   * canonical codes        Shared/huff_util.hpp:94-193
//   * MSB-first bit packing  Shared/HuffmanEncoder.cpp:211-381
//   * block bit offsets      Shared/HuffmanUtil.cpp:1103-1128
//   * split T1/T2 tables     Shared/HuffmanUtil.cpp:338-667
// No module statics (the reference keeps code tables in file statics,
// HuffmanUtil.cpp:87-102): every entry point is reentrant.
#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/metalhuffman.h"

namespace {

// Code lengths from symbol frequencies, reproducing the reference's tree
// shape exactly. The reference (HuffmanEncoder.cpp:81-102) keeps nodes in an
// array sorted by weight where a new node goes after every node whose weight
// is <= its own -- i.e. at std::upper_bound -- and build_tree (:69-79) merges
// the two front-most unconsumed entries. Leaves enter in symbol order.
int code_lengths(const uint64_t freq[256], uint8_t lens[256]) {
  std::memset(lens, 0, 256);
  struct Node { uint64_t w; int left, right; };
  std::vector<Node> nodes;
  nodes.reserve(512);
  std::vector<int> queue;  // node ids sorted by weight (stable)
  queue.reserve(512);
  auto push = [&](int id) {
    auto it = std::upper_bound(queue.begin(), queue.end(), nodes[id].w,
                               [&](uint64_t w, int other) { return w < nodes[other].w; });
    queue.insert(it, id);
  };
  int leaf_symbol[256];
  int nleaf = 0;
  for (int s = 0; s < 256; ++s) {
    if (!freq[s]) continue;
    leaf_symbol[nleaf++] = s;
    nodes.push_back({freq[s], -1, -1});
    push((int)nodes.size() - 1);
  }
  if (nleaf == 0) return MH_ERR_EMPTY;
  if (nleaf == 1) {  // single symbol -> 1-bit code "0" (HuffmanEncoder.cpp:118-121)
    lens[leaf_symbol[0]] = 1;
    return MH_OK;
  }
  size_t head = 0;
  while (head + 1 < queue.size()) {
    const int a = queue[head], b = queue[head + 1];
    head += 2;
    nodes.push_back({nodes[a].w + nodes[b].w, a, b});
    push((int)nodes.size() - 1);
  }
  // Depths top-down: internal nodes were created in order, the root last.
  std::vector<int> depth(nodes.size(), 0);
  for (int id = (int)nodes.size() - 1; id >= nleaf; --id) {
    depth[nodes[id].left] = depth[id] + 1;
    depth[nodes[id].right] = depth[id] + 1;
  }
  bool too_long = false;
  for (int i = 0; i < nleaf; ++i) {
    if (depth[i] > 16) too_long = true;
    lens[leaf_symbol[i]] = (uint8_t)std::min(depth[i], 255);
  }
  return too_long ? MH_ERR_CODE_TOO_LONG : MH_OK;
}

// huff_util.hpp:94-193: canonical order = (length, symbol); codes count up
// and are shifted left whenever the length grows; stored left-justified.
void canonical_codes(const uint8_t lens[256], uint16_t codes[256]) {
  std::memset(codes, 0, 256 * sizeof(uint16_t));
  int order[256];
  int n = 0;
  for (int s = 0; s < 256; ++s)
    if (lens[s]) order[n++] = s;
  std::stable_sort(order, order + n, [&](int a, int b) { return lens[a] < lens[b]; });
  uint32_t code = 0;
  for (int i = 0; i < n; ++i) {
    const int len = lens[order[i]];
    if (i > 0 && len > lens[order[i - 1]]) code <<= (len - lens[order[i - 1]]);
    codes[order[i]] = (uint16_t)(code << (16 - len));
    ++code;
  }
}

// MSB-first bit writer into a caller buffer.
struct BitWriter {
  uint8_t *out;
  uint64_t acc = 0;  // pending bits, right-aligned
  int nacc = 0;
  uint64_t nbytes = 0;
  uint64_t nbits = 0;
  explicit BitWriter(uint8_t *o) : out(o) {}
  inline void put(uint32_t code_lj16, int len) {
    acc = (acc << len) | (code_lj16 >> (16 - len));
    nacc += len;
    nbits += len;
    while (nacc >= 8) {
      nacc -= 8;
      out[nbytes++] = (uint8_t)(acc >> nacc);
    }
  }
  inline void flush() {  // zero-fill the last partial byte (HuffmanEncoder.cpp:279-306)
    if (nacc > 0) {
      out[nbytes++] = (uint8_t)(acc << (8 - nacc));
      nacc = 0;
    }
  }
};

int encode_symbols(const uint8_t *sym, uint64_t n, uint64_t stride, uint8_t canon[256],
                   uint8_t *codes, uint64_t codes_cap, uint64_t *codes_len, uint32_t *offsets) {
  uint64_t freq[256] = {0};
  for (uint64_t i = 0; i < n; ++i) freq[sym[i]]++;
  int rc = code_lengths(freq, canon);
  if (rc != MH_OK) return rc;
  uint16_t cc[256];
  canonical_codes(canon, cc);
  uint64_t total_bits = 0;
  for (int s = 0; s < 256; ++s) total_bits += freq[s] * canon[s];
  if (total_bits >= (1ull << 32)) return MH_ERR_CAPACITY;  // u32 block offsets
  const uint64_t need = (total_bits + 7) / 8 + 2;
  if (need > codes_cap) return MH_ERR_CAPACITY;
  BitWriter bw(codes);
  for (uint64_t i = 0; i < n; ++i) {
    if (offsets && (i % stride) == 0) offsets[i / stride] = (uint32_t)bw.nbits;
    const uint8_t s = sym[i];
    bw.put(cc[s], canon[s]);
  }
  bw.flush();
  codes[bw.nbytes++] = 0;  // decoder read-ahead (HuffmanEncoder.cpp:371-378)
  codes[bw.nbytes++] = 0;
  *codes_len = bw.nbytes;
  return MH_OK;
}

void fill_range(mh_lookup_symbol *tab, uint32_t first, uint32_t count, uint8_t sym, uint8_t len) {
  for (uint32_t i = 0; i < count; ++i) tab[first + i] = mh_lookup_symbol{sym, len};
}

}  // namespace

extern "C" {

int mh_split_blocks(const uint8_t *img, uint32_t width, uint32_t height, uint32_t block_dim,
                    uint8_t zero_value, uint8_t *out, size_t out_bytes) {
  if (!img || !out || !width || !height || !block_dim) return MH_ERR_INVALID_ARG;
  const uint32_t bw = (width + block_dim - 1) / block_dim;
  const uint32_t bh = (height + block_dim - 1) / block_dim;
  const size_t bsz = (size_t)block_dim * block_dim;
  if (out_bytes < bsz * bw * bh) return MH_ERR_CAPACITY;
  std::memset(out, zero_value, bsz * bw * bh);
  for (uint32_t by = 0; by < bh; ++by) {
    for (uint32_t bx = 0; bx < bw; ++bx) {
      uint8_t *blk = out + ((size_t)by * bw + bx) * bsz;
      const uint32_t x0 = bx * block_dim;
      const uint32_t cols = std::min(block_dim, width - x0);
      for (uint32_t r = 0; r < block_dim; ++r) {
        const uint32_t y = by * block_dim + r;
        if (y >= height) break;
        std::memcpy(blk + (size_t)r * block_dim, img + (size_t)y * width + x0, cols);
      }
    }
  }
  return MH_OK;
}

int mh_merge_blocks(const uint8_t *blocks, uint32_t width, uint32_t height, uint32_t block_dim,
                    uint8_t *out, size_t out_pitch) {
  if (!blocks || !out || !width || !height || !block_dim || out_pitch < width)
    return MH_ERR_INVALID_ARG;
  const uint32_t bw = (width + block_dim - 1) / block_dim;
  const size_t bsz = (size_t)block_dim * block_dim;
  for (uint32_t y = 0; y < height; ++y) {
    const uint32_t by = y / block_dim, r = y % block_dim;
    for (uint32_t bx = 0; bx < bw; ++bx) {
      const uint32_t x0 = bx * block_dim;
      const uint32_t cols = std::min(block_dim, width - x0);
      std::memcpy(out + (size_t)y * out_pitch + x0,
                  blocks + ((size_t)by * bw + bx) * bsz + (size_t)r * block_dim, cols);
    }
  }
  return MH_OK;
}

int mh_encode_signed_byte_deltas(const uint8_t *in, uint8_t *out, size_t n) {
  if ((!in || !out) && n) return MH_ERR_INVALID_ARG;
  uint8_t prev = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint8_t v = in[i];
    out[i] = (uint8_t)(v - prev);
    prev = v;
  }
  return MH_OK;
}

int mh_decode_signed_byte_deltas(const uint8_t *in, uint8_t *out, size_t n) {
  if ((!in || !out) && n) return MH_ERR_INVALID_ARG;
  uint8_t acc = 0;
  for (size_t i = 0; i < n; ++i) {
    acc = (uint8_t)(acc + in[i]);
    out[i] = acc;
  }
  return MH_OK;
}

uint64_t mh_codes_bound(uint64_t n_symbols) { return n_symbols * 2 + 2; }

int mh_encode_huffman(const uint8_t *symbols, uint64_t n_symbols, uint32_t block_dim,
                      uint8_t canon_header[256], uint8_t *codes, uint64_t codes_cap,
                      uint64_t *codes_len, uint32_t *block_bit_offsets) {
  if (!symbols || !canon_header || !codes || !codes_len || !block_dim) return MH_ERR_INVALID_ARG;
  if (n_symbols == 0) return MH_ERR_EMPTY;
  const uint64_t stride = (uint64_t)block_dim * block_dim;
  // HuffmanUtil.cpp:1110-1115 queries offsets only for whole blocks.
  return encode_symbols(symbols, n_symbols, stride, canon_header, codes, codes_cap, codes_len,
                        block_bit_offsets);
}

int mh_encode_frame(const uint8_t *gray, uint32_t width, uint32_t height, uint32_t flags,
                    uint8_t canon_header[256], uint8_t *codes, uint64_t codes_cap,
                    uint64_t *codes_len, uint32_t *block_offsets, uint8_t *block_init) {
  if (!gray || !canon_header || !codes || !codes_len || !block_offsets) return MH_ERR_INVALID_ARG;
  if (!width || !height || width > MH_MAX_DIM || height > MH_MAX_DIM) return MH_ERR_DIMS;
  const uint32_t bw = (width + 7) / 8, bh = (height + 7) / 8;
  const uint64_t nb = (uint64_t)bw * bh;
  std::vector<uint8_t> blocks(nb * 64);
  int rc = mh_split_blocks(gray, width, height, 8, 0, blocks.data(), blocks.size());
  if (rc != MH_OK) return rc;
  if (!(flags & MH_FLAG_NO_DELTA)) {
    for (uint64_t b = 0; b < nb; ++b) {
      uint8_t *blk = blocks.data() + b * 64;
      mh_encode_signed_byte_deltas(blk, blk, 64);
      if (block_init) {  // AAPLRenderer.m:456-472
        block_init[b] = blk[0];
        blk[0] = 0;
      }
    }
  } else if (block_init) {
    std::memset(block_init, 0, nb);  // AAPLRenderer.m:517-523
  }
  if (codes_cap < 2) return MH_ERR_CAPACITY;
  rc = encode_symbols(blocks.data(), blocks.size(), 64, canon_header, codes, codes_cap - 2,
                      codes_len, block_offsets);
  if (rc != MH_OK) return rc;
  codes[*codes_len] = 0;  // renderer read-ahead (AAPLRenderer.m:576-585)
  codes[*codes_len + 1] = 0;
  *codes_len += 2;
  return MH_OK;
}

int mh_container_header(uint64_t n_symbols, uint8_t header[MH_CONTAINER_HEADER_BYTES]) {
  if (!header) return MH_ERR_INVALID_ARG;
  if (n_symbols > 0xFFFFFFFFull) return MH_ERR_CAPACITY;
  const uint32_t words[2] = {MH_CONTAINER_MAGIC, (uint32_t)n_symbols};
  for (int w = 0; w < 2; ++w)
    for (int k = 0; k < 4; ++k) header[4 * w + k] = (uint8_t)(words[w] >> (8 * k));
  return MH_OK;
}

int mh_parse_container_header(const uint8_t header[MH_CONTAINER_HEADER_BYTES], uint64_t *n_symbols) {
  if (!header || !n_symbols) return MH_ERR_INVALID_ARG;
  uint32_t words[2] = {0, 0};
  for (int w = 0; w < 2; ++w)
    for (int k = 0; k < 4; ++k) words[w] |= (uint32_t)header[4 * w + k] << (8 * k);
  if (words[0] != MH_CONTAINER_MAGIC) return MH_ERR_INVALID_ARG;
  *n_symbols = words[1];
  return MH_OK;
}

int mh_code_lengths(const uint64_t freq[256], uint8_t canon_header[256]) {
  if (!freq || !canon_header) return MH_ERR_INVALID_ARG;
  return code_lengths(freq, canon_header);
}

int mh_canonical_codes(const uint8_t canon_header[256], uint16_t codes[256]) {
  if (!canon_header || !codes) return MH_ERR_INVALID_ARG;
  for (int s = 0; s < 256; ++s)
    if (canon_header[s] > 16) return MH_ERR_CODE_TOO_LONG;
  canonical_codes(canon_header, codes);
  return MH_OK;
}

int mh_build_tables(const uint8_t canon_header[256], mh_lookup_symbol table1[256],
                    mh_lookup_symbol *table2, uint32_t table2_cap, uint32_t *table2_entries) {
  if (!canon_header || !table1 || !table2 || !table2_entries) return MH_ERR_INVALID_ARG;
  uint16_t cc[256];
  int rc = mh_canonical_codes(canon_header, cc);
  if (rc != MH_OK) return rc;
  std::memset(table1, 0, 256 * sizeof(mh_lookup_symbol));
  // Long codes grouped by their high byte; groups numbered in ascending
  // high-byte order starting at 1 (subtable 0 is the all-zero dummy the
  // shader may read unconditionally, HuffmanUtil.cpp:550-556).
  int16_t group_of_high[256];
  std::fill(group_of_high, group_of_high + 256, (int16_t)-1);
  for (int s = 0; s < 256; ++s)
    if (canon_header[s] > 8) group_of_high[cc[s] >> 8] = 0;
  uint32_t ngroups = 0;
  for (int hp = 0; hp < 256; ++hp)
    if (group_of_high[hp] == 0) group_of_high[hp] = (int16_t)(++ngroups);
  const uint32_t entries = (ngroups + 1) * 256;
  if (entries > table2_cap) return MH_ERR_CAPACITY;
  std::memset(table2, 0, entries * sizeof(mh_lookup_symbol));
  for (int s = 0; s < 256; ++s) {
    const int len = canon_header[s];
    if (!len) continue;
    if (len <= 8) {
      fill_range(table1, cc[s] >> 8, 1u << (8 - len), (uint8_t)s, (uint8_t)len);
    } else {
      const int g = group_of_high[cc[s] >> 8];
      fill_range(table2 + (size_t)g * 256, cc[s] & 0xFF, 1u << (16 - len), (uint8_t)s,
                 (uint8_t)len);
    }
  }
  for (int hp = 0; hp < 256; ++hp)
    if (group_of_high[hp] > 0) table1[hp] = mh_lookup_symbol{(uint8_t)group_of_high[hp], 0};
  *table2_entries = entries;
  return MH_OK;
}

int mh_build_single_table(const uint8_t canon_header[256], mh_lookup_symbol table[65536]) {
  if (!canon_header || !table) return MH_ERR_INVALID_ARG;
  uint16_t cc[256];
  int rc = mh_canonical_codes(canon_header, cc);
  if (rc != MH_OK) return rc;
  std::memset(table, 0, 65536 * sizeof(mh_lookup_symbol));
  for (int s = 0; s < 256; ++s) {
    const int len = canon_header[s];
    if (len) fill_range(table, cc[s], 1u << (16 - len), (uint8_t)s, (uint8_t)len);
  }
  return MH_OK;
}

const char *mh_error_string(int status) {
  switch (status) {
    case MH_OK: return "ok";
    case MH_ERR_INVALID_ARG: return "invalid argument";
    case MH_ERR_DIMS: return "invalid dimensions";
    case MH_ERR_CODE_TOO_LONG: return "huffman code longer than 16 bits";
    case MH_ERR_CAPACITY: return "buffer too small";
    case MH_ERR_TABLE: return "invalid lookup table";
    case MH_ERR_ALIGN: return "misaligned buffer or pitch";
    case MH_ERR_HIP: return "HIP runtime error";
    case MH_ERR_EMPTY: return "no symbols";
    default: return "unknown error";
  }
}

}  // extern "C"

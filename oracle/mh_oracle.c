/*
 * mh_oracle.c -- TEST INFRASTRUCTURE ONLY (see mh_oracle.h).
 *
 * Plain-C restatement of the reference algorithm for the Huffman block codec
 * of mdejong/MetalHuffman. Written for clarity over speed: this is the checker
 * the HIP decoder is compared against, never the thing measured or shipped
 * (the cpu_baseline leg of bench.py times orc_decode_from_tables, which is the
 * reference's own CPU decode loop restated).
 */
#include "mh_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------------- */
/* Util.m:233-323 splitIntoBlocksOfSize: zero fill the whole block buffer
 * (:256), then walk image rows; row `y` lands in block row y/bdim, each block
 * of that row receives bdim bytes (fewer for the partial last column,
 * :293-302) appended after the rows already written to that block. */
int orc_split_blocks(const uint8_t *img, uint32_t w, uint32_t h, uint32_t bdim,
                     uint32_t bw, uint32_t bh, uint8_t zero, uint8_t *out) {
  if (!img || !out || bdim == 0 || bw * bdim < w || bh * bdim < h) return ORC_ERR_ARG;
  const uint32_t bsz = bdim * bdim;
  memset(out, zero, (size_t)bsz * bw * bh);
  for (uint32_t y = 0; y < h; y++) {
    const uint32_t by = y / bdim, ry = y % bdim;
    for (uint32_t bx = 0; bx < bw; bx++) {
      uint32_t x0 = bx * bdim;
      uint32_t ncopy = (x0 + bdim <= w) ? bdim : (w - x0);
      uint8_t *dst = out + (size_t)(by * bw + bx) * bsz + (size_t)ry * bdim;
      memcpy(dst, img + (size_t)y * w + x0, ncopy);
    }
  }
  return ORC_OK;
}

/* HuffmanUtil.cpp:21-47: d0 = v0, di = vi - v(i-1) (int8 wraparound). */
void orc_delta_encode(uint8_t *buf, size_t n) {
  uint8_t prev = 0;
  for (size_t i = 0; i < n; i++) {
    uint8_t v = buf[i];
    buf[i] = (uint8_t)(v - prev);
    prev = v;
  }
}

/* HuffmanUtil.cpp:49-78 (minusOne = false): vi = v(i-1) + di. */
void orc_delta_decode(uint8_t *buf, size_t n) {
  uint8_t prev = 0;
  for (size_t i = 0; i < n; i++) {
    prev = (uint8_t)(prev + buf[i]);
    buf[i] = prev;
  }
}

/* ------------------------------------------------------------------------- */
/* Tree construction, HuffmanEncoder.cpp:29-145.
 *
 * The reference keeps a 1-based node array sorted by weight. add_node
 * (:81-102) inserts a node after every node of equal or smaller weight.
 * Leaves are added in symbol order (:59-67). build_tree (:69-79) repeatedly
 * takes the next two unconsumed array slots (2k-1, 2k) and inserts their sum.
 * A code's length is the number of parent hops from the leaf to the last
 * slot (:106-145); a lone symbol gets the 1-bit code "0" (:118-121).
 * Here the array holds node ids and the tree is kept as explicit parent links.
 */
int orc_code_lengths(const uint8_t *in, uint32_t n, uint8_t canon[256]) {
  uint32_t freq[256];
  memset(freq, 0, sizeof(freq));
  for (uint32_t i = 0; i < n; i++) freq[in[i]]++;
  memset(canon, 0, 256);

  uint32_t weight[512];
  int parent[512];
  int leaf_sym[256];
  int order[513]; /* 1-based sorted array of node ids */
  int count = 0, nleaf = 0;

  for (int s = 0; s < 256; s++) {
    if (!freq[s]) continue;
    int id = nleaf++;
    leaf_sym[id] = s;
    weight[id] = freq[s];
    parent[id] = -1;
    int i = count;
    while (i > 0 && weight[order[i]] > weight[id]) { order[i + 1] = order[i]; i--; }
    order[i + 1] = id;
    count++;
  }
  if (nleaf == 0) return ORC_ERR_EMPTY;
  if (nleaf == 1) { canon[leaf_sym[0]] = 1; return ORC_OK; }

  int next_id = nleaf;
  int next_slot = 1;
  while (next_slot < count) {
    int a = order[next_slot], b = order[next_slot + 1];
    next_slot += 2;
    int id = next_id++;
    weight[id] = weight[a] + weight[b];
    parent[id] = -1;
    parent[a] = id;
    parent[b] = id;
    int i = count;
    while (i > 0 && weight[order[i]] > weight[id]) { order[i + 1] = order[i]; i--; }
    order[i + 1] = id;
    count++;
  }
  int too_long = 0;
  for (int id = 0; id < nleaf; id++) {
    int depth = 0;
    for (int p = parent[id]; p >= 0; p = parent[p]) depth++;
    if (depth > 16) too_long = 1;
    canon[leaf_sym[id]] = (uint8_t)depth;
  }
  return too_long ? ORC_ERR_TOO_LONG : ORC_OK;
}

/* huff_util.hpp:94-193: order symbols by (length, symbol); the code counter
 * starts at 0, is stored left-justified in 16 bits, incremented, and shifted
 * left by the length increase before the next (longer) symbol. */
void orc_canonical_codes(const uint8_t canon[256], uint16_t codes[256]) {
  memset(codes, 0, 256 * sizeof(uint16_t));
  uint32_t code = 0;
  int prev_len = 0;
  for (int len = 1; len <= 16; len++) {
    for (int s = 0; s < 256; s++) {
      if (canon[s] != len) continue;
      if (prev_len && len > prev_len) code <<= (len - prev_len);
      prev_len = len;
      codes[s] = (uint16_t)((code << (16 - len)) & 0xFFFF);
      code++;
    }
  }
}

/* HuffmanEncoder.cpp:211-306 + :310-381: MSB-first packing, per-symbol bit
 * offsets (:229), zero-filled last byte (:279-306), 2 zero bytes (:377-378);
 * HuffmanUtil.cpp:1108-1117: offsets of symbols 0, stride, 2*stride, ... */
int orc_huffman_encode(const uint8_t *in, uint32_t n, uint32_t stride,
                       uint8_t canon[256], uint8_t *codes, uint64_t codes_cap,
                       uint64_t *codes_len, uint32_t *offsets) {
  int rc = orc_code_lengths(in, n, canon);
  if (rc != ORC_OK) return rc;
  uint16_t cc[256];
  orc_canonical_codes(canon, cc);
  uint64_t bit = 0;
  uint64_t nbytes_needed = 0;
  for (uint32_t i = 0; i < n; i++) nbytes_needed += canon[in[i]];
  nbytes_needed = (nbytes_needed + 7) / 8 + 2;
  if (nbytes_needed > codes_cap) return ORC_ERR_CAP;
  memset(codes, 0, nbytes_needed);
  for (uint32_t i = 0; i < n; i++) {
    if (offsets && stride && (i % stride) == 0) offsets[i / stride] = (uint32_t)bit;
    const uint8_t s = in[i];
    const int len = canon[s];
    for (int k = 0; k < len; k++, bit++) {
      if ((cc[s] >> (15 - k)) & 1) codes[bit >> 3] |= (uint8_t)(0x80u >> (bit & 7));
    }
  }
  *codes_len = nbytes_needed;
  return ORC_OK;
}

/* ------------------------------------------------------------------------- */
/* HuffmanUtil.cpp:116-265 generateLookupTableRange: every table slot whose
 * index starts with the symbol's (shifted, masked) code bits gets {sym, len}. */
static void fill_prefix(orc_sym *tab, uint32_t prefix_bits, int free_bits, uint8_t sym,
                        uint8_t len) {
  const uint32_t count = 1u << free_bits;
  for (uint32_t g = 0; g < count; g++) {
    tab[prefix_bits | g].symbol = sym;
    tab[prefix_bits | g].bitWidth = len;
  }
}

/* HuffmanUtil.cpp:338-667 generateSplitLookupTables(8, 8): short codes
 * (len <= 8) fill T1 directly (:383-412); long codes are grouped by their
 * high 8 bits (:441-497); T2 holds one dummy all-zero subtable followed by
 * one 256-entry subtable per group in ascending high-prefix order
 * (:530-620); T1[high] = {subtable index, 0} (:631-646). */
int orc_split_tables(const uint8_t canon[256], orc_sym t1[256], orc_sym *t2,
                     uint32_t t2_cap, uint32_t *t2_entries) {
  uint16_t cc[256];
  orc_canonical_codes(canon, cc);
  memset(t1, 0, 256 * sizeof(orc_sym));
  for (int s = 0; s < 256; s++) {
    const int len = canon[s];
    if (len < 1 || len > 8) continue;
    fill_prefix(t1, (uint32_t)(cc[s] >> 8), 8 - len, (uint8_t)s, (uint8_t)len);
  }
  int has_group[256];
  memset(has_group, 0, sizeof(has_group));
  for (int s = 0; s < 256; s++)
    if (canon[s] > 8) has_group[cc[s] >> 8] = 1;
  uint32_t ngroups = 0;
  for (int hp = 0; hp < 256; hp++) ngroups += has_group[hp];
  const uint32_t entries = (ngroups + 1) * 256;
  if (entries > t2_cap) return ORC_ERR_CAP;
  memset(t2, 0, entries * sizeof(orc_sym));
  uint32_t sub = 1;
  for (int hp = 0; hp < 256; hp++) {
    if (!has_group[hp]) continue;
    orc_sym *tab = t2 + (size_t)sub * 256;
    for (int s = 0; s < 256; s++) {
      const int len = canon[s];
      if (len <= 8 || (cc[s] >> 8) != hp) continue;
      fill_prefix(tab, (uint32_t)(cc[s] & 0xFF), 16 - len, (uint8_t)s, (uint8_t)len);
    }
    t1[hp].symbol = (uint8_t)sub;
    t1[hp].bitWidth = 0;
    sub++;
  }
  *t2_entries = entries;
  return ORC_OK;
}

/* HuffmanUtil.cpp:314-334 generateLookupTable over the full 16-bit range. */
int orc_single_table(const uint8_t canon[256], orc_sym t[65536]) {
  uint16_t cc[256];
  orc_canonical_codes(canon, cc);
  memset(t, 0, 65536 * sizeof(orc_sym));
  for (int s = 0; s < 256; s++) {
    const int len = canon[s];
    if (!len) continue;
    if (len > 16) return ORC_ERR_TOO_LONG;
    fill_prefix(t, cc[s], 16 - len, (uint8_t)s, (uint8_t)len);
  }
  return ORC_OK;
}

/* ------------------------------------------------------------------------- */
/* The 16-bit window at absolute bit position `pos`, built from 3 bytes the way
 * HuffmanUtil.cpp:866-947 and AAPLShaders.metal:137-155 do it. */
static inline uint32_t window16(const uint8_t *buf, uint64_t pos) {
  const uint64_t nb = pos >> 3;
  const uint32_t m = (uint32_t)(pos & 7);
  uint32_t b0 = buf[nb], b1 = buf[nb + 1], b2 = buf[nb + 2];
  b0 = ((b0 << m) & 0xFF) << 8;
  b1 = b1 << m;
  b2 = b2 >> (8 - m);
  return (b0 | b1 | b2) & 0xFFFF;
}

/* HuffmanUtil.cpp:961-995 / AAPLShaders.metal:159-170. */
static inline orc_sym lookup_split(const orc_sym *t1, const orc_sym *t2, uint32_t pat) {
  orc_sym e = t1[pat >> 8];
  if (e.bitWidth == 0) e = t2[(uint32_t)e.symbol * 256u + (pat & 0xFF)];
  return e;
}

void orc_decode_from_tables(const orc_sym *t1, const orc_sym *t2, uint32_t nsym,
                            const uint8_t *buf, uint8_t *out, uint32_t *bit_offsets) {
  uint64_t pos = 0;
  for (uint32_t i = 0; i < nsym; i++) {
    const orc_sym e = lookup_split(t1, t2, window16(buf, pos));
    if (bit_offsets) bit_offsets[i] = (uint32_t)pos;
    out[i] = e.symbol;
    pos += e.bitWidth;
  }
}

void orc_decode_single_table(const orc_sym *t, uint32_t nsym, const uint8_t *buf,
                             uint8_t *out, uint32_t *bit_offsets) {
  uint64_t pos = 0;
  for (uint32_t i = 0; i < nsym; i++) {
    const orc_sym e = t[window16(buf, pos)];
    if (bit_offsets) bit_offsets[i] = (uint32_t)pos;
    out[i] = e.symbol;
    pos += e.bitWidth;
  }
}

/* AAPLShaders.metal:241-268 + :291-445: per block, 64 serial steps from
 * root = offsets[blocki] with a u16 running bit count and a u16 prev symbol,
 * prev = (prev + sym) & 0xFF; :449-518: pixel (x, y) reads symbol
 * k = (y%8)*8 + x%8 of block (x/8, y/8); output cropped to W x H. */
int orc_decode_frame_shader(const uint32_t *block_offsets, const uint8_t *codes,
                            const orc_sym *t1, const orc_sym *t2, uint32_t w,
                            uint32_t h, uint32_t bw, uint32_t bh,
                            const uint8_t *block_init, int delta, uint8_t *out) {
  if (bw * 8 < w || bh * 8 < h) return ORC_ERR_ARG;
  uint8_t blk[64];
  for (uint32_t by = 0; by < bh; by++) {
    for (uint32_t bx = 0; bx < bw; bx++) {
      const uint32_t bi = by * bw + bx;
      const uint32_t root = block_offsets[bi];
      uint16_t nread = 0;
      uint16_t prev = block_init ? block_init[bi] : 0;
      for (int k = 0; k < 64; k++) {
        const uint64_t cur = (uint64_t)root + nread;
        const orc_sym e = lookup_split(t1, t2, window16(codes, cur));
        nread = (uint16_t)(nread + e.bitWidth);
        if (delta) {
          prev = (uint16_t)((prev + e.symbol) & 0xFF);
          blk[k] = (uint8_t)prev;
        } else {
          blk[k] = e.symbol;
        }
      }
      for (uint32_t ry = 0; ry < 8; ry++) {
        const uint32_t y = by * 8 + ry;
        if (y >= h) break;
        for (uint32_t rx = 0; rx < 8; rx++) {
          const uint32_t x = bx * 8 + rx;
          if (x >= w) break;
          out[(size_t)y * w + x] = blk[ry * 8 + rx];
        }
      }
    }
  }
  return ORC_OK;
}

/* The decode contract's debug report (the product's mh_check):
 * per block, the same 64 steps as AAPLShaders.metal:241-268, counting
 * report[0] zero-width lookups ({0,0} entries, HuffmanUtil.cpp:550-556),
 * report[1] T1 escapes to a subtable at/after t2_entries (counted as zero width),
 * report[2] blocks (all but the last) whose codes end off the next block's offset,
 * report[3] first offending block or 0xFFFFFFFF. Bytes past codes_bytes read 0. */
void orc_check_frame(const uint32_t *block_offsets, const uint8_t *codes, uint64_t codes_bytes,
                     const orc_sym *t1, const orc_sym *t2, uint32_t t2_entries, uint32_t nb,
                     uint32_t report[4]) {
  report[0] = report[1] = report[2] = 0;
  report[3] = 0xFFFFFFFFu;
  for (uint32_t b = 0; b < nb; b++) {
    uint64_t pos = block_offsets[b];
    uint32_t zw = 0, esc = 0;
    for (int k = 0; k < 64; k++) {
      const uint64_t i = pos >> 3;
      const uint32_t m = (uint32_t)(pos & 7);
      const uint32_t b0 = i < codes_bytes ? codes[i] : 0;
      const uint32_t b1 = i + 1 < codes_bytes ? codes[i + 1] : 0;
      const uint32_t b2 = i + 2 < codes_bytes ? codes[i + 2] : 0;
      const uint32_t pat = ((((b0 << m) & 0xFF) << 8) | (b1 << m) | (b2 >> (8 - m))) & 0xFFFF;
      orc_sym e = t1[pat >> 8];
      if (e.bitWidth == 0) {
        const uint32_t idx = (uint32_t)e.symbol * 256u + (pat & 0xFF);
        if (idx < t2_entries) {
          e = t2[idx];
        } else {
          esc++;
          e.symbol = 0;
          e.bitWidth = 0;
        }
      }
      if (e.bitWidth == 0) zw++;
      pos += e.bitWidth;
    }
    const int mism = b + 1 < nb && pos != block_offsets[b + 1];
    if (zw || esc || mism) {
      report[0] += zw;
      report[1] += esc;
      report[2] += (uint32_t)mism;
      if (b < report[3]) report[3] = b;
    }
  }
}

/* AAPLRenderer.m:374-688 (setupHuffmanEncoding) for blockDim 8, deltas on. */
int orc_encode_frame(const uint8_t *img, uint32_t w, uint32_t h, uint8_t canon[256],
                     uint8_t *codes, uint64_t codes_cap, uint64_t *codes_len,
                     uint32_t *block_offsets) {
  const uint32_t bw = (w + 7) / 8, bh = (h + 7) / 8;
  const size_t n = (size_t)bw * bh * 64;
  uint8_t *blocks = (uint8_t *)malloc(n);
  if (!blocks) return ORC_ERR_CAP;
  int rc = orc_split_blocks(img, w, h, 8, bw, bh, 0, blocks);
  if (rc == ORC_OK) {
    for (size_t b = 0; b < (size_t)bw * bh; b++) orc_delta_encode(blocks + b * 64, 64);
    if (codes_cap < 2) rc = ORC_ERR_CAP;
    else rc = orc_huffman_encode(blocks, (uint32_t)n, 64, canon, codes, codes_cap - 2,
                                 codes_len, block_offsets);
  }
  if (rc == ORC_OK) {
    codes[*codes_len] = 0;
    codes[*codes_len + 1] = 0;
    *codes_len += 2;
  }
  free(blocks);
  return rc;
}

/* ------------------------------------------------------------------------- */
typedef struct {
  const orc_sym *t1, *t2;
  uint32_t nsym;
  const uint8_t *const *bufs;
  uint8_t *const *outs;
  uint32_t n_frames, n_threads, tid, reps;
  uint32_t w, h;      /* pipeline mode: raster size (0: symbols only) */
  uint8_t *scratch;   /* pipeline mode: nsym block-order symbols per thread */
} orc_job;

/* Block-order deltas -> W x H raster: the per-block prefix sum
 * (HuffmanUtil::decodeSignedByteDeltas, HuffmanUtil.cpp:49-78, per 64-symbol block as
 * the renderer's producer step delta-encodes per block, AAPLRenderer.m:374-688) and the
 * block merge (Util.m:233-323's inverse: block (bx, by) row r -> raster row 8 by + r). */
static void undelta_raster(uint8_t *sym, uint32_t w, uint32_t h, uint8_t *raster) {
  const uint32_t bw = (w + 7) / 8, bh = (h + 7) / 8;
  for (uint32_t b = 0; b < bw * bh; b++) orc_delta_decode(sym + (size_t)b * 64, 64);
  for (uint32_t y = 0; y < h; y++) {
    const uint32_t by = y / 8, ry = y % 8;
    for (uint32_t bx = 0; bx < bw; bx++) {
      const uint32_t x0 = bx * 8, n = x0 + 8 <= w ? 8 : w - x0;
      memcpy(raster + (size_t)y * w + x0, sym + ((size_t)(by * bw + bx) * 64 + ry * 8), n);
    }
  }
}

static void *decode_worker(void *arg) {
  orc_job *j = (orc_job *)arg;
  for (uint32_t r = 0; r < j->reps; r++)
    for (uint32_t f = j->tid; f < j->n_frames; f += j->n_threads) {
      if (j->w) {
        orc_decode_from_tables(j->t1, j->t2, j->nsym, j->bufs[f], j->scratch, NULL);
        undelta_raster(j->scratch, j->w, j->h, j->outs[f]);
      } else {
        orc_decode_from_tables(j->t1, j->t2, j->nsym, j->bufs[f], j->outs[f], NULL);
      }
    }
  return NULL;
}

static double time_jobs(const orc_sym *t1, const orc_sym *t2, uint32_t nsym,
                        const uint8_t *const *bufs, uint8_t *const *outs, uint32_t n_frames,
                        uint32_t n_threads, uint32_t reps, uint32_t w, uint32_t h) {
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 1024) n_threads = 1024;
  pthread_t *th = (pthread_t *)calloc(n_threads, sizeof(pthread_t));
  orc_job *jobs = (orc_job *)calloc(n_threads, sizeof(orc_job));
  if (!th || !jobs) {
    free(th);
    free(jobs);
    return -1.0;
  }
  for (uint32_t t = 0; t < n_threads; t++) {
    jobs[t] = (orc_job){t1, t2, nsym, bufs, outs, n_frames, n_threads, t, reps, w, h, NULL};
    if (w) jobs[t].scratch = (uint8_t *)malloc(nsym);
  }
  struct timespec t0, t1c;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (uint32_t t = 0; t < n_threads; t++) pthread_create(&th[t], NULL, decode_worker, &jobs[t]);
  for (uint32_t t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1c);
  for (uint32_t t = 0; t < n_threads; t++) free(jobs[t].scratch);
  free(th);
  free(jobs);
  return (double)(t1c.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1c.tv_nsec - t0.tv_nsec);
}

double orc_time_decode_frames(const orc_sym *t1, const orc_sym *t2, uint32_t nsym,
                              const uint8_t *const *bufs, uint8_t *const *outs,
                              uint32_t n_frames, uint32_t n_threads, uint32_t reps) {
  return time_jobs(t1, t2, nsym, bufs, outs, n_frames, n_threads, reps, 0, 0);
}

double orc_time_decode_pipeline(const orc_sym *t1, const orc_sym *t2, uint32_t w, uint32_t h,
                                const uint8_t *const *bufs, uint8_t *const *rasters,
                                uint32_t n_frames, uint32_t n_threads, uint32_t reps) {
  const uint32_t nsym = ((w + 7) / 8) * ((h + 7) / 8) * 64;
  return time_jobs(t1, t2, nsym, bufs, rasters, n_frames, n_threads, reps, w, h);
}

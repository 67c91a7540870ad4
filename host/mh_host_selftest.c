/* mh_host_selftest.c -- round trips and garbage inputs through the host half of the C-ABI
 * (mh_host.cpp, mh_cpu.cpp: the producer and the CPU decoders), meant to be built with
 * the host compiler's AddressSanitizer and UndefinedBehaviorSanitizer
 * (tests/test_host_sanitize.py). No GPU and no HIP: it links the two host sources only.
 *
 * Per case (size, picture kind, format):
 *   encode (mh_encode_frame) -> tables (mh_build_tables) -> mh_decode_frame_cpu on 1 and
 *   3 threads == the picture; the same symbols through the split / delta / mh_encode_huffman
 *   steps, decoded by mh_decode_huffman_bits_from_tables and mh_decode_huffman_bits (the
 *   single 64K table) == the symbols; the container header round trip. Then the frame's
 *   code bytes and block offsets are scrambled and decoded again: the result is not
 *   checked (garbage in), only that every access stays inside the caller's buffers, as
 *   the header promises ("bytes past codes_bytes read as zero").
 * Prints one line per failure and "selftest ok <cases>" at the end; exit status 0 iff ok. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/metalhuffman.h"

static uint64_t rng_state;
static uint32_t rnd(void) {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 7;
  rng_state ^= rng_state << 17;
  return (uint32_t)(rng_state >> 11);
}

/* kinds: 0 smooth gradient + small noise (skewed deltas, long tail), 1 uniform random
 * bytes (flat 8-bit code), 2 constant (one symbol), 3 two levels, 4 Fibonacci-skewed
 * noise (codes up to 16 bits, sometimes more: those cases are skipped) */
static void make_picture(uint8_t *img, uint32_t w, uint32_t h, int kind) {
  for (uint32_t y = 0; y < h; ++y)
    for (uint32_t x = 0; x < w; ++x) {
      uint8_t v;
      switch (kind) {
        case 0: v = (uint8_t)((x * 3 + y * 5) / 7 + (rnd() % 5)); break;
        case 1: v = (uint8_t)rnd(); break;
        case 2: v = 77; break;
        case 3: v = (rnd() & 1) ? 10 : 200; break;
        default: {
          uint32_t r = rnd(), k = 0;
          while (k < 20 && (r & 1)) { r >>= 1; ++k; }
          v = (uint8_t)(k * 11);
        }
      }
      img[(size_t)y * w + x] = v;
    }
}

static int failures = 0;
#define FAIL(...)                      \
  do {                                 \
    fprintf(stderr, __VA_ARGS__);      \
    fputc('\n', stderr);               \
    ++failures;                        \
  } while (0)

static void one_case(uint32_t w, uint32_t h, int kind, uint32_t flags, int with_init) {
  const uint32_t bw = (w + 7) / 8, bh = (h + 7) / 8;
  const uint64_t nb = (uint64_t)bw * bh, n = nb * 64;
  uint8_t *img = malloc((size_t)w * h);
  make_picture(img, w, h, kind);
  const uint64_t cap = mh_codes_bound(n) + 2;
  uint8_t *codes = malloc(cap);
  uint32_t *offsets = malloc(nb * 4);
  uint8_t *init = with_init ? malloc(nb) : NULL;
  uint8_t canon[256];
  uint64_t codes_len = 0;
  int rc = mh_encode_frame(img, w, h, flags, canon, codes, cap, &codes_len, offsets, init);
  if (rc == MH_ERR_CODE_TOO_LONG) goto done;  /* the reference asserts here too */
  if (rc != MH_OK) { FAIL("%ux%u kind %d: mh_encode_frame %d", w, h, kind, rc); goto done; }
  {
    mh_lookup_symbol t1[256];
    mh_lookup_symbol *t2 = malloc(sizeof(mh_lookup_symbol) * MH_TABLE2_MAX_ENTRIES);
    uint32_t t2e = 0;
    rc = mh_build_tables(canon, t1, t2, MH_TABLE2_MAX_ENTRIES, &t2e);
    if (rc != MH_OK) { FAIL("%ux%u kind %d: mh_build_tables %d", w, h, kind, rc); free(t2); goto done; }
    uint8_t *out = malloc((size_t)w * h);
    for (uint32_t threads = 1; threads <= 3; threads += 2) {
      memset(out, 0xA5, (size_t)w * h);
      rc = mh_decode_frame_cpu(offsets, codes, codes_len, t1, t2, t2e, init, w, h, flags, out, w, threads);
      if (rc != MH_OK || memcmp(out, img, (size_t)w * h) != 0)
        FAIL("%ux%u kind %d flags %u init %d threads %u: frame decode rc %d or bytes differ", w, h, kind, flags,
             with_init, threads, rc);
    }
    /* the producer's steps one by one, and both serial CPU decoders */
    uint8_t *blocks = malloc(n), *sym = malloc(n), *dec = malloc(n);
    rc = mh_split_blocks(img, w, h, 8, 0, blocks, n);
    if (rc == MH_OK) rc = mh_encode_signed_byte_deltas(blocks, sym, n);
    uint8_t canon2[256];
    uint8_t *codes2 = malloc(cap);
    uint32_t *off2 = malloc(nb * 4);
    uint64_t len2 = 0;
    if (rc == MH_OK) rc = mh_encode_huffman(sym, n, 8, canon2, codes2, cap, &len2, off2);
    if (rc == MH_OK) {
      mh_lookup_symbol t1b[256];
      uint32_t t2eb = 0;
      rc = mh_build_tables(canon2, t1b, t2, MH_TABLE2_MAX_ENTRIES, &t2eb);
      if (rc == MH_OK)
        rc = mh_decode_huffman_bits_from_tables(t1b, t2, t2eb, 8, 8, n, codes2, len2, dec, NULL);
      if (rc != MH_OK || memcmp(dec, sym, n) != 0) FAIL("%ux%u kind %d: split-table decode rc %d or differs", w, h, kind, rc);
      mh_lookup_symbol *single = malloc(sizeof(mh_lookup_symbol) * 65536);
      uint32_t *bits = malloc(n * 4);
      rc = mh_build_single_table(canon2, single);
      if (rc == MH_OK) rc = mh_decode_huffman_bits(single, n, codes2, len2, dec, bits);
      if (rc != MH_OK || memcmp(dec, sym, n) != 0) FAIL("%ux%u kind %d: single-table decode rc %d or differs", w, h, kind, rc);
      for (uint64_t b = 0; b < nb && rc == MH_OK; ++b)
        if (bits[b * 64] != off2[b]) { FAIL("%ux%u kind %d: block %llu offset", w, h, kind, (unsigned long long)b); break; }
      if (mh_decode_signed_byte_deltas(sym, dec, n) != MH_OK || memcmp(dec, blocks, n) != 0)
        FAIL("%ux%u kind %d: delta round trip", w, h, kind);
      free(single);
      free(bits);
    } else if (rc != MH_ERR_CODE_TOO_LONG) {
      FAIL("%ux%u kind %d: producer steps rc %d", w, h, kind, rc);
    }
    uint8_t hdr[MH_CONTAINER_HEADER_BYTES];
    uint64_t back = 0;
    if (mh_container_header(n, hdr) != MH_OK || mh_parse_container_header(hdr, &back) != MH_OK || back != n)
      FAIL("container header round trip %llu", (unsigned long long)n);
    /* garbage in: scrambled code bytes, then scrambled offsets (any bit inside the
     * payload), then offsets far past it -- only memory safety is checked */
    for (uint64_t i = 0; i + MH_CODES_PAD < codes_len; ++i) codes[i] = (uint8_t)rnd();
    (void)mh_decode_frame_cpu(offsets, codes, codes_len, t1, t2, t2e, init, w, h, flags, out, w, 2);
    for (uint64_t b = 0; b < nb; ++b) offsets[b] = (uint32_t)(rnd() % (uint32_t)(codes_len * 8));
    (void)mh_decode_frame_cpu(offsets, codes, codes_len, t1, t2, t2e, init, w, h, flags, out, w, 1);
    for (uint64_t b = 0; b < nb; ++b) offsets[b] = 0xFFFFFF00u - (uint32_t)b;
    (void)mh_decode_frame_cpu(offsets, codes, codes_len, t1, t2, t2e, init, w, h, flags, out, w, 1);
    (void)mh_decode_huffman_bits_from_tables(t1, t2, t2e, 8, 8, n, codes, codes_len, dec, NULL);
    free(blocks);
    free(sym);
    free(dec);
    free(codes2);
    free(off2);
    free(out);
    free(t2);
  }
done:
  free(img);
  free(codes);
  free(offsets);
  free(init);
}

int main(int argc, char **argv) {
  rng_state = argc > 1 ? strtoull(argv[1], NULL, 10) | 1u : 0x9E3779B97F4A7C15ull;
  static const uint32_t dims[][2] = {{1, 1}, {7, 9}, {8, 8}, {9, 7}, {64, 64}, {333, 517}, {1000, 8}, {3, 1001}, {512, 384}};
  int cases = 0;
  for (size_t d = 0; d < sizeof(dims) / sizeof(dims[0]); ++d)
    for (int kind = 0; kind < 5; ++kind) {
      one_case(dims[d][0], dims[d][1], kind, 0, 0);
      one_case(dims[d][0], dims[d][1], kind, MH_FLAG_NO_DELTA, 0);
      one_case(dims[d][0], dims[d][1], kind, 0, 1);
      cases += 3;
    }
  if (failures) {
    printf("selftest FAILED %d of %d\n", failures, cases);
    return 1;
  }
  printf("selftest ok %d\n", cases);
  return 0;
}

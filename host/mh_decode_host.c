/* mh_decode_host.c -- the "small C host" of the drop-in boundary: a plain C
 * program that drives the MI355X decoder through the C-ABI in
 * include/metalhuffman.h and the HIP runtime's C API, the way the reference's
 * renderer drives its Metal passes (Shared/AAPLRenderer.m:374-688 setup,
 * :1178-1678 per frame). No Python, no torch.
 *
 *   mh_decode_host synth W H [reps]
 *       deterministic synthetic W x H frame: host encode (mh_encode_frame), tables
 *       (mh_build_tables), upload, mh_prepare_lut, mh_decode, verify, time.
 *   mh_decode_host raw W H file.gray [reps]
 *       the same for an 8-bit raw image file.
 *   mh_decode_host buffers W H canon.bin codes.bin offsets.bin expected.gray
 *       buffers exactly as the reference encoder emits them (256-byte canonical
 *       header, MSB-first codes, u32 LE block bit offsets -- HuffmanUtil.cpp:
 *       1051-1131) decoded unchanged and compared with the expected pixels.
 *   mh_decode_host device W H [reps]
 *       the whole chain on the GPU with no host round trip: the frame is encoded
 *       on the device (mh_encode_frame_device_async), the tables are built from
 *       the device header (mh_build_tables_device), then mh_decode; the encoded
 *       bytes are compared with the host codec's and the raster with the frame.
 *
 * Prints one line "decode ok W H ..." (exit 0) or the first mismatch (exit 1).
 */
#define _POSIX_C_SOURCE 199309L /* clock_gettime under -std=c11 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "metalhuffman.h"

#define HIP_OK(x)                                                        \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      fprintf(stderr, "%s:%d: %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(2);                                                           \
    }                                                                    \
  } while (0)

#define MH_OK_OR_DIE(x)                                                  \
  do {                                                                   \
    int rc_ = (x);                                                       \
    if (rc_ != MH_OK) {                                                  \
      fprintf(stderr, "%s:%d: %s\n", __FILE__, __LINE__, mh_error_string(rc_)); \
      exit(2);                                                           \
    }                                                                    \
  } while (0)

static void *xmalloc(size_t n) {
  void *p = calloc(1, n ? n : 1);
  if (!p) {
    fprintf(stderr, "out of memory (%zu bytes)\n", n);
    exit(2);
  }
  return p;
}

static uint8_t *read_file(const char *path, size_t *len) {
  FILE *f = fopen(path, "rb");
  if (!f) {
    fprintf(stderr, "cannot open %s\n", path);
    exit(2);
  }
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t *buf = (uint8_t *)xmalloc((size_t)n + MH_CODES_PAD);
  if (n > 0 && fread(buf, 1, (size_t)n, f) != (size_t)n) {
    fprintf(stderr, "short read %s\n", path);
    exit(2);
  }
  fclose(f);
  *len = (size_t)n;
  return buf;
}

/* smooth gradient plus small noise: a natural-image-like delta histogram */
static void synth_frame(uint8_t *img, uint32_t w, uint32_t h) {
  uint32_t s = 12345u;
  for (uint32_t y = 0; y < h; ++y)
    for (uint32_t x = 0; x < w; ++x) {
      s = s * 1664525u + 1013904223u;
      img[(size_t)y * w + x] = (uint8_t)((x / 3 + y / 5 + ((s >> 24) & 7u)) & 0xFFu);
    }
}

/* encode -> tables -> decode, all on the device (the producer and the consumer of
 * the reference's buffers on one GPU, nothing through the host in between) */
static int device_chain(uint32_t w, uint32_t h, int reps) {
  const uint32_t bw = (w + 7) / 8, bh = (h + 7) / 8, nb = bw * bh;
  const size_t pitch = ((size_t)w + 7) & ~(size_t)7;
  uint8_t *img = (uint8_t *)xmalloc((size_t)w * h);
  synth_frame(img, w, h);
  /* the host codec's bytes, to compare with */
  const uint64_t cap = mh_codes_bound((uint64_t)nb * 64) + MH_CODES_PAD + 4;
  uint8_t canon[256], *codes = (uint8_t *)xmalloc(cap);
  uint32_t *offsets = (uint32_t *)xmalloc((size_t)nb * 4);
  uint64_t codes_len = 0;
  MH_OK_OR_DIE(mh_encode_frame(img, w, h, 0, canon, codes, cap, &codes_len, offsets, NULL));

  uint8_t *d_gray, *d_codes, *d_canon, *d_out, *d_ws;
  uint32_t *d_offsets, *d_t2_entries;
  uint64_t *d_codes_len;
  int32_t *d_status;
  mh_lookup_symbol *d_t1, *d_t2;
  uint16_t *d_lut;
  const size_t ws = mh_encode_workspace_bytes(w, h);
  HIP_OK(hipMalloc((void **)&d_gray, (size_t)w * h));
  HIP_OK(hipMalloc((void **)&d_codes, cap));
  HIP_OK(hipMalloc((void **)&d_canon, 256));
  HIP_OK(hipMalloc((void **)&d_out, pitch * h));
  HIP_OK(hipMalloc((void **)&d_ws, ws));
  HIP_OK(hipMalloc((void **)&d_offsets, (size_t)nb * 4));
  HIP_OK(hipMalloc((void **)&d_t2_entries, 4));
  HIP_OK(hipMalloc((void **)&d_codes_len, 8));
  HIP_OK(hipMalloc((void **)&d_status, 8));
  HIP_OK(hipMalloc((void **)&d_t1, 256 * sizeof(mh_lookup_symbol)));
  HIP_OK(hipMalloc((void **)&d_t2, MH_TABLE2_MAX_ENTRIES * sizeof(mh_lookup_symbol)));
  HIP_OK(hipMalloc((void **)&d_lut, mh_lut_bytes()));
  HIP_OK(hipMemcpy(d_gray, img, (size_t)w * h, hipMemcpyHostToDevice));

  mh_frame fr;
  memset(&fr, 0, sizeof(fr));
  fr.d_block_offsets = d_offsets;
  fr.d_codes = d_codes;
  fr.codes_bytes = cap; /* the byte count stays on the device: the decoder bounds blocks by offsets */
  fr.d_table1 = d_t1;
  fr.d_table2 = d_t2;
  fr.table2_entries = MH_TABLE2_MAX_ENTRIES;
  fr.d_lut = d_lut;
  fr.dims.width = w;
  fr.dims.height = h;
  fr.dims.block_width = bw;
  fr.dims.block_height = bh;
  fr.n_frames = 1;

#define CHAIN()                                                                                      \
  do {                                                                                               \
    MH_OK_OR_DIE(mh_encode_frame_device_async(d_gray, w, h, 0, d_canon, d_codes, cap, d_codes_len,   \
                                              d_offsets, NULL, d_status, d_ws, ws, NULL));           \
    MH_OK_OR_DIE(mh_build_tables_device(d_canon, d_t1, d_t2, d_t2_entries, d_lut, d_status + 1, NULL)); \
    MH_OK_OR_DIE(mh_decode(&fr, d_out, pitch, pitch * h, NULL));                                     \
  } while (0)
  CHAIN();
  HIP_OK(hipDeviceSynchronize());
  int32_t status[2];
  uint64_t dev_len = 0;
  uint8_t dev_canon[256];
  HIP_OK(hipMemcpy(status, d_status, 8, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(&dev_len, d_codes_len, 8, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(dev_canon, d_canon, 256, hipMemcpyDeviceToHost));
  if (status[0] != MH_OK || status[1] != MH_OK) {
    printf("device status %d %d\n", status[0], status[1]);
    return 1;
  }
  uint8_t *dev_codes = (uint8_t *)xmalloc(codes_len);
  uint32_t *dev_offsets = (uint32_t *)xmalloc((size_t)nb * 4);
  HIP_OK(hipMemcpy(dev_codes, d_codes, codes_len, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(dev_offsets, d_offsets, (size_t)nb * 4, hipMemcpyDeviceToHost));
  if (dev_len != codes_len || memcmp(dev_canon, canon, 256) || memcmp(dev_codes, codes, codes_len) ||
      memcmp(dev_offsets, offsets, (size_t)nb * 4)) {
    printf("ENCODE MISMATCH: device %llu bytes vs host %llu\n", (unsigned long long)dev_len,
           (unsigned long long)codes_len);
    return 1;
  }
  uint8_t *got = (uint8_t *)xmalloc(pitch * h);
  HIP_OK(hipMemcpy(got, d_out, pitch * h, hipMemcpyDeviceToHost));
  for (uint32_t y = 0; y < h; ++y)
    for (uint32_t x = 0; x < w; ++x)
      if (got[(size_t)y * pitch + x] != img[(size_t)y * w + x]) {
        printf("MISMATCH at x=%u y=%u\n", x, y);
        return 1;
      }
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  HIP_OK(hipEventRecord(e0, NULL));
  for (int i = 0; i < reps; ++i) CHAIN();
  HIP_OK(hipEventRecord(e1, NULL));
  HIP_OK(hipEventSynchronize(e1));
  float ms = 0.f;
  HIP_OK(hipEventElapsedTime(&ms, e0, e1));
#undef CHAIN
  printf("device ok %u %u codes_bytes %llu us_per_encode_tables_decode %.2f\n", w, h,
         (unsigned long long)codes_len, reps > 0 ? 1e3 * ms / reps : 0.0);
  hipFree(d_gray);
  hipFree(d_codes);
  hipFree(d_canon);
  hipFree(d_out);
  hipFree(d_ws);
  hipFree(d_offsets);
  hipFree(d_t2_entries);
  hipFree(d_codes_len);
  hipFree(d_status);
  hipFree(d_t1);
  hipFree(d_t2);
  hipFree(d_lut);
  free(img);
  free(codes);
  free(offsets);
  free(dev_codes);
  free(dev_offsets);
  free(got);
  return 0;
}

int main(int argc, char **argv) {
  if (argc < 4) {
    fprintf(stderr,
            "usage: %s synth W H [reps] | raw W H file.gray [reps] |\n"
            "       buffers W H canon.bin codes.bin offsets.bin expected.gray | device W H [reps]\n",
            argv[0]);
    return 2;
  }
  const char *mode = argv[1];
  const uint32_t w = (uint32_t)strtoul(argv[2], NULL, 10), h = (uint32_t)strtoul(argv[3], NULL, 10);
  const uint32_t bw = (w + 7) / 8, bh = (h + 7) / 8, nb = bw * bh;
  int reps = 20;
  if (!strcmp(mode, "device")) return device_chain(w, h, argc > 4 ? atoi(argv[4]) : 20);

  uint8_t canon[256];
  uint8_t *codes = NULL, *expected = NULL;
  uint32_t *offsets = NULL;
  uint64_t codes_len = 0; /* bytes incl. the MH_CODES_PAD zero bytes */

  if (!strcmp(mode, "synth") || !strcmp(mode, "raw")) {
    expected = (uint8_t *)xmalloc((size_t)w * h);
    if (!strcmp(mode, "synth")) {
      synth_frame(expected, w, h);
      if (argc > 4) reps = atoi(argv[4]);
    } else {
      size_t n = 0;
      uint8_t *img = read_file(argv[4], &n);
      if (n != (size_t)w * h) {
        fprintf(stderr, "raw file holds %zu bytes, expected %u\n", n, w * h);
        return 2;
      }
      memcpy(expected, img, n);
      free(img);
      if (argc > 5) reps = atoi(argv[5]);
    }
    /* the renderer's producer step (AAPLRenderer.m:374-688) */
    const uint64_t cap = mh_codes_bound((uint64_t)nb * 64) + MH_CODES_PAD;
    codes = (uint8_t *)xmalloc(cap);
    offsets = (uint32_t *)xmalloc((size_t)nb * 4);
    MH_OK_OR_DIE(mh_encode_frame(expected, w, h, 0, canon, codes, cap, &codes_len, offsets, NULL));
  } else if (!strcmp(mode, "buffers") && argc >= 8) {
    size_t n = 0;
    uint8_t *c = read_file(argv[4], &n);
    if (n != 256) {
      fprintf(stderr, "canonical header must be 256 bytes\n");
      return 2;
    }
    memcpy(canon, c, 256);
    free(c);
    size_t cl = 0;
    codes = read_file(argv[5], &cl); /* + MH_CODES_PAD zero bytes (read_file) */
    codes_len = cl + 2;              /* the renderer's 2 extra bytes (AAPLRenderer.m:576-585) */
    size_t ol = 0;
    offsets = (uint32_t *)read_file(argv[6], &ol);
    if (ol != (size_t)nb * 4) {
      fprintf(stderr, "offsets file holds %zu bytes, expected %u\n", ol, nb * 4);
      return 2;
    }
    size_t el = 0;
    expected = read_file(argv[7], &el);
    if (el != (size_t)w * h) {
      fprintf(stderr, "expected image holds %zu bytes, expected %u\n", el, w * h);
      return 2;
    }
  } else {
    fprintf(stderr, "unknown mode %s\n", mode);
    return 2;
  }

  /* tables (parseCanonicalHeader + generateSplitLookupTables, AAPLRenderer.m:568-608) */
  mh_lookup_symbol t1[256];
  mh_lookup_symbol *t2 = (mh_lookup_symbol *)xmalloc(sizeof(mh_lookup_symbol) * MH_TABLE2_MAX_ENTRIES);
  uint32_t t2_entries = 0;
  MH_OK_OR_DIE(mh_build_tables(canon, t1, t2, MH_TABLE2_MAX_ENTRIES, &t2_entries));

  /* device buffers (the renderer's MTLBuffers, AAPLRenderer.m:582, 657-667, 863) */
  const size_t pitch = ((size_t)w + 7) & ~(size_t)7;
  uint8_t *d_codes, *d_out;
  uint32_t *d_offsets;
  mh_lookup_symbol *d_t1, *d_t2;
  uint16_t *d_lut;
  HIP_OK(hipMalloc((void **)&d_codes, codes_len));
  HIP_OK(hipMalloc((void **)&d_offsets, (size_t)nb * 4));
  HIP_OK(hipMalloc((void **)&d_t1, sizeof(t1)));
  HIP_OK(hipMalloc((void **)&d_t2, sizeof(mh_lookup_symbol) * t2_entries));
  HIP_OK(hipMalloc((void **)&d_lut, mh_lut_bytes()));
  HIP_OK(hipMalloc((void **)&d_out, pitch * h));
  HIP_OK(hipMemcpy(d_codes, codes, codes_len, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_offsets, offsets, (size_t)nb * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_t1, t1, sizeof(t1), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_t2, t2, sizeof(mh_lookup_symbol) * t2_entries, hipMemcpyHostToDevice));
  MH_OK_OR_DIE(mh_prepare_lut(d_t1, d_t2, t2_entries, d_lut, NULL));

  mh_frame fr;
  memset(&fr, 0, sizeof(fr));
  fr.d_block_offsets = d_offsets;
  fr.d_codes = d_codes;
  fr.codes_bytes = codes_len;
  fr.d_table1 = d_t1;
  fr.d_table2 = d_t2;
  fr.table2_entries = t2_entries;
  fr.d_lut = d_lut;
  fr.dims.width = w;
  fr.dims.height = h;
  fr.dims.block_width = bw;
  fr.dims.block_height = bh;
  fr.n_frames = 1;

  /* optional debug check of the buffers (mh_check), then one decode + verify */
  uint32_t *d_report, report[4];
  HIP_OK(hipMalloc((void **)&d_report, sizeof(report)));
  MH_OK_OR_DIE(mh_check(&fr, d_report, NULL));
  HIP_OK(hipMemcpy(report, d_report, sizeof(report), hipMemcpyDeviceToHost));
  MH_OK_OR_DIE(mh_decode(&fr, d_out, pitch, pitch * h, NULL));
  HIP_OK(hipDeviceSynchronize());
  uint8_t *got = (uint8_t *)xmalloc(pitch * h);
  HIP_OK(hipMemcpy(got, d_out, pitch * h, hipMemcpyDeviceToHost));
  for (uint32_t y = 0; y < h; ++y)
    for (uint32_t x = 0; x < w; ++x)
      if (got[(size_t)y * pitch + x] != expected[(size_t)y * w + x]) {
        printf("MISMATCH at x=%u y=%u: got %u expected %u\n", x, y, got[(size_t)y * pitch + x],
               expected[(size_t)y * w + x]);
        return 1;
      }

  /* timing: reps back-to-back launches between two events; the host's own time per
     mh_decode call (what a per-frame caller pays on the CPU) beside it */
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  HIP_OK(hipEventRecord(e0, NULL));
  struct timespec h0, h1;
  clock_gettime(CLOCK_MONOTONIC, &h0);
  for (int i = 0; i < reps; ++i) MH_OK_OR_DIE(mh_decode(&fr, d_out, pitch, pitch * h, NULL));
  clock_gettime(CLOCK_MONOTONIC, &h1);
  HIP_OK(hipEventRecord(e1, NULL));
  HIP_OK(hipEventSynchronize(e1));
  float ms = 0.f;
  HIP_OK(hipEventElapsedTime(&ms, e0, e1));
  const double us = reps > 0 ? 1e3 * ms / reps : 0.0;
  const double host_us =
      reps > 0 ? ((double)(h1.tv_sec - h0.tv_sec) * 1e6 + (double)(h1.tv_nsec - h0.tv_nsec) * 1e-3) / reps : 0.0;
  printf("decode ok %u %u codes_bytes %llu t2_entries %u check %u %u %u us_per_launch %.2f MBps %.1f "
         "host_us_per_call %.2f\n",
         w, h, (unsigned long long)codes_len, t2_entries, report[0], report[1], report[2], us,
         us > 0 ? (double)w * h / us : 0.0, host_us);

  hipFree(d_codes);
  hipFree(d_offsets);
  hipFree(d_t1);
  hipFree(d_t2);
  hipFree(d_lut);
  hipFree(d_out);
  hipFree(d_report);
  free(codes);
  free(offsets);
  free(expected);
  free(got);
  free(t2);
  return 0;
}

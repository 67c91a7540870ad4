/* mh_decode_multi.c -- the multi-GPU path from the plain-C host (VERDICT r03 item 6;
 * SURVEY.md 8(e); north_star: "driven from a small C host over a thin C-ABI",
 * "RCCL broadcast of the shared symbol table over xGMI only").
 *
 * The reference renders on ONE command queue (Shared/AAPLRenderer.m:996); frames are
 * independent, so N GPUs each decode their own shard with no exchange on the data
 * path. One host thread per device (the C-ABI keeps no global state: each thread
 * drives its own device and stream):
 *
 *   1. the table: device 0 encodes the base frame on the GPU
 *      (mh_encode_frame_device_async) and its 256-byte canonical header is
 *      broadcast from device 0 to every device with ncclBroadcast over one RCCL
 *      communicator per device (ncclCommInitAll; xGMI between the GPUs of a node);
 *      every device builds T1/T2 and its decode table from the header
 *      (mh_build_tables_device) -- parseCanonicalHeader + generateSplitLookupTables,
 *      HuffmanUtil.cpp:270-667, on the device;
 *   2. the shard: device d holds frames [d F, (d + 1) F), 8x8-block shuffles of the
 *      base frame (one shared histogram, so one table); they are uploaded and
 *      encoded on the device in one batched call (mh_encode_frames_device_async),
 *      each frame's header checked against the broadcast one;
 *   3. the decode: `reps` batch launches of all F frames (mh_decode), timed with HIP
 *      events per device and with the wall clock across devices (threads meet at a
 *      barrier before and after; wall = slowest device), then every decoded raster
 *      compared with its input frame on the host.
 *
 *   mh_decode_multi N F [reps] [W H file.gray]
 *       N devices (<= hipGetDeviceCount), F frames per device per launch; the base
 *       frame is the raw W x H file (e.g. BigBridge) or a synthetic 2048 x 1536 one.
 *
 * Prints one line per device (its HIP ordinal and PCI bus id; the ids must be distinct),
 * then one line "multi ok N ... devices_verified N" (exit 0), or the failures (exit 1 / 2).
 */
#define _POSIX_C_SOURCE 200809L
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "metalhuffman.h"

#define HIP_OK(x)                                                                      \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d: %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
      exit(2);                                                                         \
    }                                                                                  \
  } while (0)
#define MH_OK_OR_DIE(x)                                                                \
  do {                                                                                 \
    int rc_ = (x);                                                                     \
    if (rc_ != MH_OK) {                                                                \
      fprintf(stderr, "%s:%d: %s\n", __FILE__, __LINE__, mh_error_string(rc_));        \
      exit(2);                                                                         \
    }                                                                                  \
  } while (0)
#define NCCL_OK(x)                                                                     \
  do {                                                                                 \
    ncclResult_t r_ = (x);                                                             \
    if (r_ != ncclSuccess) {                                                           \
      fprintf(stderr, "%s:%d: %s\n", __FILE__, __LINE__, ncclGetErrorString(r_));      \
      exit(2);                                                                         \
    }                                                                                  \
  } while (0)

enum { kMaxDevices = 64 };

typedef struct {
  int dev, n_dev, n_frames, reps;
  uint32_t w, h;
  const uint8_t *base;        /* the base frame (host) */
  ncclComm_t comm;
  pthread_barrier_t *bar;
  double *walls;              /* [0] before, [1] after the timed region (thread 0 writes) */
  /* results */
  float us_per_launch;
  int ok;
  char msg[256];
  char pci[64];               /* the device's PCI bus id (hipDeviceGetPCIBusId) */
} Worker;

static void *xmalloc(size_t n) {
  void *p = calloc(1, n ? n : 1);
  if (!p) {
    fprintf(stderr, "out of memory (%zu bytes)\n", n);
    exit(2);
  }
  return p;
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* smooth gradient plus small noise (as mh_decode_host's synthetic frame) */
static void synth_frame(uint8_t *img, uint32_t w, uint32_t h) {
  uint32_t s = 12345u;
  for (uint32_t y = 0; y < h; ++y)
    for (uint32_t x = 0; x < w; ++x) {
      s = s * 1664525u + 1013904223u;
      img[(size_t)y * w + x] = (uint8_t)((x / 3 + y / 5 + ((s >> 24) & 7u)) & 0xFFu);
    }
}

/* frame `seed`: the base frame's 8x8 blocks permuted (Fisher-Yates, xorshift64*);
 * W and H are multiples of 8, so every block is whole and the delta histogram -- hence
 * the canonical table -- is the base frame's */
static void block_shuffle(const uint8_t *src, uint8_t *dst, uint32_t w, uint32_t h, uint64_t seed) {
  const uint32_t bw = w / 8, nb = bw * (h / 8);
  uint32_t *perm = (uint32_t *)xmalloc((size_t)nb * 4);
  for (uint32_t i = 0; i < nb; ++i) perm[i] = i;
  uint64_t x = seed * 0x9E3779B97F4A7C15ull + 0x2545F4914F6CDD1Dull;
  for (uint32_t i = nb - 1; i > 0; --i) {
    x ^= x >> 12, x ^= x << 25, x ^= x >> 27;
    const uint32_t j = (uint32_t)(((x * 0x2545F4914F6CDD1Dull) >> 32) % (i + 1));
    const uint32_t t = perm[i];
    perm[i] = perm[j];
    perm[j] = t;
  }
  for (uint32_t b = 0; b < nb; ++b) {
    const uint32_t s = perm[b];
    const uint32_t sx = (s % bw) * 8, sy = (s / bw) * 8, dx = (b % bw) * 8, dy = (b / bw) * 8;
    for (uint32_t r = 0; r < 8; ++r) memcpy(dst + (size_t)(dy + r) * w + dx, src + (size_t)(sy + r) * w + sx, 8);
  }
  free(perm);
}

static void *worker(void *arg) {
  Worker *k = (Worker *)arg;
  const uint32_t w = k->w, h = k->h, bw = w / 8, bh = h / 8, nb = bw * bh;
  const int F = k->n_frames;
  const size_t px = (size_t)w * h, pitch = w;
  HIP_OK(hipSetDevice(k->dev));
  HIP_OK(hipDeviceGetPCIBusId(k->pci, (int)sizeof(k->pci), k->dev));
  hipStream_t st;
  HIP_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));

  /* 1. the shared table: device 0's GPU encoder makes the header, RCCL broadcasts it */
  uint8_t *d_canon;
  HIP_OK(hipMalloc((void **)&d_canon, 256));
  if (k->dev == 0) {
    uint8_t *d_gray, *d_codes, *d_ws;
    uint32_t *d_offs;
    const uint64_t cap = mh_codes_bound((uint64_t)nb * 64) + MH_CODES_PAD + 16;
    const size_t ws = mh_encode_workspace_bytes(w, h);
    HIP_OK(hipMalloc((void **)&d_gray, px));
    HIP_OK(hipMalloc((void **)&d_codes, cap));
    HIP_OK(hipMalloc((void **)&d_ws, ws));
    HIP_OK(hipMalloc((void **)&d_offs, (size_t)nb * 4));
    HIP_OK(hipMemcpyAsync(d_gray, k->base, px, hipMemcpyHostToDevice, st));
    MH_OK_OR_DIE(mh_encode_frame_device_async(d_gray, w, h, 0, d_canon, d_codes, cap, NULL, d_offs, NULL, NULL,
                                              d_ws, ws, st));
    HIP_OK(hipStreamSynchronize(st));
    hipFree(d_gray), hipFree(d_codes), hipFree(d_ws), hipFree(d_offs);
  }
  NCCL_OK(ncclBroadcast(d_canon, d_canon, 256, ncclUint8, 0, k->comm, st));
  mh_lookup_symbol *d_t1, *d_t2;
  uint32_t *d_t2n;
  uint16_t *d_lut;
  int32_t *d_status;
  HIP_OK(hipMalloc((void **)&d_t1, 256 * sizeof(mh_lookup_symbol)));
  HIP_OK(hipMalloc((void **)&d_t2, MH_TABLE2_MAX_ENTRIES * sizeof(mh_lookup_symbol)));
  HIP_OK(hipMalloc((void **)&d_t2n, 4));
  HIP_OK(hipMalloc((void **)&d_lut, mh_lut_bytes()));
  HIP_OK(hipMalloc((void **)&d_status, 4 * (size_t)(F + 1)));
  MH_OK_OR_DIE(mh_build_tables_device(d_canon, d_t1, d_t2, d_t2n, d_lut, d_status + F, st));

  /* 2. this device's shard, uploaded and encoded on the device in one batched call */
  uint8_t *frames = (uint8_t *)xmalloc(px * (size_t)F);
  for (int f = 0; f < F; ++f) block_shuffle(k->base, frames + px * f, w, h, (uint64_t)(k->dev * F + f));
  const uint64_t slot = ((mh_codes_bound((uint64_t)nb * 64) + MH_CODES_PAD + 15) / 16) * 16;
  const size_t bws = mh_encode_frames_workspace_bytes(w, h, (uint32_t)F);
  uint8_t *d_gray, *d_codes, *d_canons, *d_ws, *d_out;
  uint32_t *d_offs;
  uint64_t *d_fco;
  HIP_OK(hipMalloc((void **)&d_gray, px * F));
  HIP_OK(hipMalloc((void **)&d_codes, slot * F));
  HIP_OK(hipMalloc((void **)&d_canons, 256 * (size_t)F));
  HIP_OK(hipMalloc((void **)&d_ws, bws));
  HIP_OK(hipMalloc((void **)&d_offs, (size_t)nb * 4 * F));
  HIP_OK(hipMalloc((void **)&d_fco, 8 * (size_t)(F + 1)));
  HIP_OK(hipMalloc((void **)&d_out, px * F));
  HIP_OK(hipMemcpyAsync(d_gray, frames, px * F, hipMemcpyHostToDevice, st));
  MH_OK_OR_DIE(mh_encode_frames_device_async(d_gray, px, (uint32_t)F, w, h, 0, d_canons, d_codes, slot, NULL, d_fco,
                                             d_offs, NULL, d_status, d_ws, bws, st));
  int32_t *status = (int32_t *)xmalloc(4 * (size_t)(F + 1));
  uint8_t *canons = (uint8_t *)xmalloc(256 * (size_t)F), canon[256];
  HIP_OK(hipMemcpyAsync(status, d_status, 4 * (size_t)(F + 1), hipMemcpyDeviceToHost, st));
  HIP_OK(hipMemcpyAsync(canons, d_canons, 256 * (size_t)F, hipMemcpyDeviceToHost, st));
  HIP_OK(hipMemcpyAsync(canon, d_canon, 256, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  k->ok = 1;
  for (int f = 0; f <= F && k->ok; ++f)
    if (status[f] != MH_OK) {
      snprintf(k->msg, sizeof(k->msg), "device %d: status %d (%s)", k->dev, status[f], f < F ? "encode" : "tables");
      k->ok = 0;
    }
  for (int f = 0; f < F && k->ok; ++f)
    if (memcmp(canons + 256 * (size_t)f, canon, 256)) {
      snprintf(k->msg, sizeof(k->msg), "device %d frame %d: header differs from the broadcast one", k->dev, f);
      k->ok = 0;
    }

  /* 3. reps batch launches of the shard, timed */
  mh_frame fr;
  memset(&fr, 0, sizeof(fr));
  fr.d_block_offsets = d_offs;
  fr.d_codes = d_codes;
  fr.codes_bytes = slot * F;
  fr.d_frame_code_offsets = d_fco;
  fr.d_table1 = d_t1;
  fr.d_table2 = d_t2;
  fr.table2_entries = MH_TABLE2_MAX_ENTRIES;
  fr.d_lut = d_lut;
  fr.dims.width = w;
  fr.dims.height = h;
  fr.dims.block_width = bw;
  fr.dims.block_height = bh;
  fr.n_frames = (uint32_t)F;
  /* A rejected shard (a frame's encode status, a header that differs from the
   * broadcast one, the table build) is never decoded: its offsets / slots were not
   * written or do not match the tables. Its thread still meets the others at both
   * barriers, so no device blocks, and reports FAIL without timing numbers. */
  if (k->ok) {
    MH_OK_OR_DIE(mh_decode(&fr, d_out, pitch, px, st)); /* warm-up */
    HIP_OK(hipStreamSynchronize(st));
  }
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  pthread_barrier_wait(k->bar);
  if (k->dev == 0) k->walls[0] = now_s();
  HIP_OK(hipEventRecord(e0, st));
  if (k->ok)
    for (int r = 0; r < k->reps; ++r) MH_OK_OR_DIE(mh_decode(&fr, d_out, pitch, px, st));
  HIP_OK(hipEventRecord(e1, st));
  HIP_OK(hipStreamSynchronize(st));
  pthread_barrier_wait(k->bar);
  if (k->dev == 0) k->walls[1] = now_s();
  float ms = 0.f;
  HIP_OK(hipEventElapsedTime(&ms, e0, e1));
  k->us_per_launch = k->reps && k->ok ? 1e3f * ms / (float)k->reps : 0.f;

  /* every decoded raster against its input frame */
  uint8_t *got = (uint8_t *)xmalloc(px * F);
  if (k->ok) HIP_OK(hipMemcpy(got, d_out, px * F, hipMemcpyDeviceToHost));
  for (int f = 0; f < F && k->ok; ++f)
    if (memcmp(got + px * f, frames + px * f, px)) {
      snprintf(k->msg, sizeof(k->msg), "device %d frame %d: decoded raster differs from the input", k->dev, f);
      k->ok = 0;
    }
  hipFree(d_canon), hipFree(d_t1), hipFree(d_t2), hipFree(d_t2n), hipFree(d_lut), hipFree(d_status);
  hipFree(d_gray), hipFree(d_codes), hipFree(d_canons), hipFree(d_ws), hipFree(d_offs), hipFree(d_fco);
  hipFree(d_out);
  hipEventDestroy(e0), hipEventDestroy(e1), hipStreamDestroy(st);
  free(frames), free(status), free(canons), free(got);
  return NULL;
}

int main(int argc, char **argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s N F [reps] [W H file.gray]\n", argv[0]);
    return 2;
  }
  const int n = atoi(argv[1]), F = atoi(argv[2]), reps = argc > 3 ? atoi(argv[3]) : 20;
  uint32_t w = 2048, h = 1536;
  uint8_t *base;
  if (argc > 6) {
    w = (uint32_t)strtoul(argv[4], NULL, 10);
    h = (uint32_t)strtoul(argv[5], NULL, 10);
    FILE *fp = fopen(argv[6], "rb");
    if (!fp) {
      fprintf(stderr, "cannot open %s\n", argv[6]);
      return 2;
    }
    base = (uint8_t *)xmalloc((size_t)w * h);
    if (fread(base, 1, (size_t)w * h, fp) != (size_t)w * h) {
      fprintf(stderr, "%s holds fewer than %u x %u bytes\n", argv[6], w, h);
      return 2;
    }
    fclose(fp);
  } else {
    base = (uint8_t *)xmalloc((size_t)w * h);
    synth_frame(base, w, h);
  }
  int avail = 0;
  HIP_OK(hipGetDeviceCount(&avail));
  if (n < 1 || n > avail || n > kMaxDevices || F < 1 || reps < 0 || w % 8 || h % 8) {
    fprintf(stderr, "need 1 <= N <= %d devices, F >= 1, W and H multiples of 8\n", avail);
    return 2;
  }
  int devs[kMaxDevices];
  ncclComm_t comms[kMaxDevices];
  for (int d = 0; d < n; ++d) devs[d] = d;
  NCCL_OK(ncclCommInitAll(comms, n, devs));
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, (unsigned)n);
  double walls[2] = {0, 0};
  Worker *ws = (Worker *)xmalloc(sizeof(Worker) * (size_t)n);
  pthread_t th[kMaxDevices];
  for (int d = 0; d < n; ++d) {
    ws[d] = (Worker){.dev = d, .n_dev = n, .n_frames = F, .reps = reps, .w = w, .h = h, .base = base,
                     .comm = comms[d], .bar = &bar, .walls = walls};
    if (pthread_create(&th[d], NULL, worker, &ws[d])) {
      fprintf(stderr, "pthread_create failed\n");
      return 2;
    }
  }
  for (int d = 0; d < n; ++d) pthread_join(th[d], NULL);
  int ok = 1;
  float worst = 0.f;
  /* self-proving multi-GPU run: each worker's HIP ordinal and PCI bus id; N distinct
   * bus ids mean N physical GPUs took part (not one GPU visible N times) */
  int distinct = 1;
  for (int d = 0; d < n; ++d) {
    printf("device %d ordinal %d pci %s us_per_launch %.2f %s\n", d, ws[d].dev, ws[d].pci, ws[d].us_per_launch,
           ws[d].ok ? "ok" : "FAIL");
    for (int e = 0; e < d; ++e)
      if (!strcmp(ws[d].pci, ws[e].pci)) distinct = 0;
  }
  if (!distinct) {
    printf("FAIL devices do not have distinct PCI bus ids\n");
    ok = 0;
  }
  for (int d = 0; d < n; ++d) {
    if (!ws[d].ok) {
      printf("FAIL %s\n", ws[d].msg);
      ok = 0;
    }
    if (ws[d].us_per_launch > worst) worst = ws[d].us_per_launch;
  }
  for (int d = 0; d < n; ++d) ncclCommDestroy(comms[d]);
  pthread_barrier_destroy(&bar);
  if (!ok) return 1;
  const double wall_us = (walls[1] - walls[0]) * 1e6 / (reps ? reps : 1);
  const double pixels = (double)w * h * F * n;
  printf("multi ok %d devices %d frames_per_device %u %u reps %d broadcast_bytes 256 worst_device_us_per_launch "
         "%.2f wall_us_per_launch %.2f MBps_events %.1f MBps_wall %.1f devices_verified %d\n",
         n, F, w, h, reps, worst, wall_us, worst > 0 ? pixels / worst : 0.0, wall_us > 0 ? pixels / wall_us : 0.0, n);
  free(ws);
  free(base);
  return 0;
}

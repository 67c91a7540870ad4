// stream_group_mock.cpp -- CPU test harness for the stream group's member and device
// bookkeeping (metalhuffman_amd/csrc/mh_stream.cpp, compiled unchanged beside this
// file with g++). The HIP runtime calls it makes are replaced by fakes that keep a
// "current device" per thread and record, for every copy and decode, which device
// was current and which device the stream belongs to; mh_decode is a fake too. The
// program then checks what tests/test_stream_group_host.py asks of it and exits 0.
//
// Reference behaviour being extended: one command queue, one device
// (Shared/AAPLRenderer.m:996, 1178-1921); the group round-robins frames over devices.
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/metalhuffman.h"

namespace {
int g_ndev = 4;
thread_local int g_cur = 0;
int g_set_calls = 0;
struct FakeStream {
  int device;
};
struct Op {
  char kind;  // 'c' copy, 'd' decode (eager), 'g' graph launch
  int cur;    // device current at the call
  int owner;  // device the stream was created on
  const void *dst;
};
std::vector<Op> g_ops;
std::vector<FakeStream *> g_streams;
int g_fail = 0;
#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "CHECK failed line %d: %s\n", __LINE__, #c); \
      ++g_fail;                                                       \
    }                                                                 \
  } while (0)
int owner_of(hipStream_t s) { return s ? reinterpret_cast<FakeStream *>(s)->device : -1; }
}  // namespace

extern "C" {
hipError_t hipGetDevice(int *d) {
  *d = g_cur;
  return hipSuccess;
}
hipError_t hipSetDevice(int d) {
  if (d < 0 || d >= g_ndev) return hipErrorInvalidDevice;
  g_cur = d;
  ++g_set_calls;
  return hipSuccess;
}
hipError_t hipGetDeviceCount(int *n) {
  *n = g_ndev;
  return hipSuccess;
}
hipError_t hipMalloc(void **p, size_t n) {
  *p = std::calloc(1, n ? n : 1);
  return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void *p) {
  std::free(p);
  return hipSuccess;
}
hipError_t hipMemset(void *p, int v, size_t n) {
  std::memset(p, v, n);
  return hipSuccess;
}
hipError_t hipMemcpyAsync(void *dst, const void *src, size_t n, hipMemcpyKind, hipStream_t s) {
  std::memcpy(dst, src, n);
  g_ops.push_back({'c', g_cur, owner_of(s), dst});
  return hipSuccess;
}
hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned int) {
  FakeStream *f = new FakeStream{g_cur};
  g_streams.push_back(f);
  *s = reinterpret_cast<hipStream_t>(f);
  return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) {
  CHECK(owner_of(s) == g_cur);  // destroyed with its own device current
  return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t s) {
  CHECK(owner_of(s) == g_cur);
  return hipSuccess;
}
hipError_t hipDeviceSynchronize(void) { return hipSuccess; }
hipError_t hipEventCreate(hipEvent_t *e) {
  *e = reinterpret_cast<hipEvent_t>(new int(g_cur));
  return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t e) {
  delete reinterpret_cast<int *>(e);
  return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t, hipStream_t s) {
  CHECK(owner_of(s) == g_cur);
  return hipSuccess;
}
hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
hipError_t hipEventElapsedTime(float *ms, hipEvent_t, hipEvent_t) {
  *ms = 0.f;
  return hipSuccess;
}
hipError_t hipStreamBeginCapture(hipStream_t, hipStreamCaptureMode) { return hipSuccess; }
hipError_t hipStreamEndCapture(hipStream_t s, hipGraph_t *g) {
  *g = reinterpret_cast<hipGraph_t>(new int(owner_of(s)));
  return hipSuccess;
}
hipError_t hipGraphInstantiate(hipGraphExec_t *x, hipGraph_t g, hipGraphNode_t *, char *, size_t) {
  *x = reinterpret_cast<hipGraphExec_t>(new int(*reinterpret_cast<int *>(g)));
  return hipSuccess;
}
hipError_t hipGraphLaunch(hipGraphExec_t x, hipStream_t s) {
  CHECK(*reinterpret_cast<int *>(x) == owner_of(s));  // the slot's graph on the slot's stream
  g_ops.push_back({'g', g_cur, owner_of(s), nullptr});
  return hipSuccess;
}
hipError_t hipGraphDestroy(hipGraph_t g) {
  delete reinterpret_cast<int *>(g);
  return hipSuccess;
}
hipError_t hipGraphExecDestroy(hipGraphExec_t x) {
  delete reinterpret_cast<int *>(x);
  return hipSuccess;
}
int mh_decode(const mh_frame *f, uint8_t *out, size_t, size_t, void *s) {
  CHECK(f && out && f->n_frames == 1 && f->d_frame_code_offsets == nullptr);
  g_ops.push_back({'d', g_cur, owner_of((hipStream_t)s), out});
  return MH_OK;
}
}  // extern "C"

int main() {
  // members on devices 2, 0, 2, 1 (a device may hold several members); the caller
  // works on device 3 throughout and must find it current after every call
  const int devices[4] = {2, 0, 2, 1};
  const uint32_t W = 64, H = 24, nb = (W / 8) * (H / 8);
  mh_frame protos[4] = {};
  uint8_t t1[512] = {}, t2[512] = {};
  for (auto &p : protos) {
    p.d_table1 = reinterpret_cast<const mh_lookup_symbol *>(t1);
    p.d_table2 = reinterpret_cast<const mh_lookup_symbol *>(t2);
    p.table2_entries = 256;
    p.dims = {W, H, W / 8, H / 8};
    p.n_frames = 1;
  }
  g_cur = 3;
  mh_stream_group *g = nullptr;
  CHECK(mh_stream_group_create(protos, 4, devices, 1024, 2, &g) == MH_OK && g);
  CHECK(g_cur == 3);
  CHECK(mh_stream_group_size(g) == 4);
  // each member's stream lives on its device
  for (uint32_t m = 0; m < 4; ++m) CHECK(mh_stream_device(mh_stream_group_member(g, m)) == devices[m]);
  CHECK(mh_stream_group_member(g, 4) == nullptr);
  // bad device ordinals are refused before anything is created
  const int bad[2] = {0, 7};
  mh_stream_group *g2 = nullptr;
  CHECK(mh_stream_group_create(protos, 2, bad, 1024, 2, &g2) == MH_ERR_INVALID_ARG && !g2);
  CHECK(g_cur == 3);

  std::vector<uint8_t> host(((nb * 4 + 15) & ~15u) + 256, 0);
  const uint32_t *offs = reinterpret_cast<const uint32_t *>(host.data());
  const uint8_t *codes = host.data() + ((nb * 4 + 15) & ~15u);
  g_ops.clear();
  for (uint32_t i = 0; i < 10; ++i) {
    uint32_t member = 99, slot = 99;
    const size_t before = g_ops.size();
    CHECK(mh_stream_group_submit(g, codes, 64, offs, nullptr, &member, &slot) == MH_OK);
    CHECK(member == i % 4);            // round robin over members
    CHECK(slot == (i / 4) % 2);        // each member alternates its two slots
    CHECK(g_cur == 3);                 // the caller's device restored
    // every copy and decode of this submit ran on the member's device, on one of its streams
    CHECK(g_ops.size() > before);
    for (size_t k = before; k < g_ops.size(); ++k) {
      CHECK(g_ops[k].cur == devices[member]);
      CHECK(g_ops[k].owner == devices[member]);
    }
    // the submit's copy landed in that member's slot buffer
    size_t pitch = 0;
    CHECK(mh_stream_output(mh_stream_group_member(g, member), slot, &pitch) != nullptr && pitch == W);
  }
  CHECK(mh_stream_group_synchronize(g) == MH_OK);
  CHECK(g_cur == 3);
  CHECK(mh_stream_group_destroy(g) == MH_OK);
  CHECK(g_cur == 3);
  std::printf("ops %zu set_device_calls %d failures %d\n", g_ops.size(), g_set_calls, g_fail);
  return g_fail ? 1 : 0;
}

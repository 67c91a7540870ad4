// mh_stream.cpp -- frames streamed from host memory (BASELINE config 5, SURVEY.md
// 8(f) rank 2): the native analogue of the reference's per-frame command buffer
// (Shared/AAPLRenderer.m:1178-1921, one decode per drawInMTKView).
//
// A stream owns `slots` device slots (codes, block offsets, optional per-block
// init bytes, output raster), each with its own HIP stream. mh_stream_submit
// copies one frame's host buffers into the next slot (hipMemcpyAsync; pinned host
// memory makes it a DMA) and replays that slot's captured decode graph, both on
// the slot's stream: the copy of frame i+1 (next slot, next stream) overlaps the
// decode of frame i, and stream order alone keeps a slot's previous decode ahead
// of the copy that reuses it -- no cross-stream event per frame. (A copy stream
// plus a compute stream needed an event record and a cross-stream wait at each
// hand-off and sustained 16.2 K frames/s; per-slot streams 20.8-21.3 K, the rate
// of bare back-to-back copies: profiles/r01_v17_stream_slots.txt.) A slot's output
// stays valid until `slots` further submits.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/metalhuffman.h"

struct mh_stream {
  struct Slot {
    uint8_t *base = nullptr;    // [block offsets, padded to 16 B][codes]
    uint8_t *codes = nullptr;
    uint32_t *offsets = nullptr;
    uint8_t *init = nullptr;
    uint8_t *out = nullptr;
    bool own_out = true;
    hipEvent_t start = nullptr;  // before the slot's copy (timing event)
    hipEvent_t done = nullptr;   // after the slot's decode (timing event)
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    hipStream_t stream = nullptr;  // this slot's copies + decode, in order
    bool used = false;
  };
  int device = 0;
  uint32_t last = 0;  // slot of the most recent submit
  mh_frame proto{};
  uint64_t cap = 0;
  uint64_t nb = 0;
  uint64_t off_bytes = 0;  // nb * 4 rounded up to 16
  size_t pitch = 0, out_bytes = 0;
  uint32_t next = 0;
  bool graphs = true;
  std::vector<Slot> slots;
};

namespace {

// Makes `dev` current for the scope (and restores the caller's device): every
// stream call may come from any host thread with any current device.
struct DeviceGuard {
  int prev = -1;
  bool ok = true;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) {
      ok = false;
      return;
    }
    if (prev != dev && hipSetDevice(dev) != hipSuccess) ok = false;
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

void release(mh_stream *s) {
  if (!s) return;
  for (auto &sl : s->slots) {
    if (sl.exec) (void)hipGraphExecDestroy(sl.exec);
    if (sl.graph) (void)hipGraphDestroy(sl.graph);
    if (sl.done) (void)hipEventDestroy(sl.done);
    if (sl.start) (void)hipEventDestroy(sl.start);
    if (sl.stream) (void)hipStreamDestroy(sl.stream);
    (void)hipFree(sl.base);
    (void)hipFree(sl.init);
    if (sl.own_out) (void)hipFree(sl.out);
  }
  delete s;
}

bool decode_slot(mh_stream *s, mh_stream::Slot &sl, hipStream_t st) {
  mh_frame f = s->proto;
  f.d_codes = sl.codes;
  f.codes_bytes = s->cap;
  f.d_block_offsets = sl.offsets;
  f.d_block_init = sl.init;
  return mh_decode(&f, sl.out, s->pitch, s->out_bytes, st) == MH_OK;
}

}  // namespace

extern "C" {

int mh_stream_create(const mh_frame *proto, uint64_t codes_capacity, uint32_t n_slots,
                     uint8_t *const *d_outputs, mh_stream **out) {
  if (!proto || !out || !proto->d_table1 || !proto->d_table2 || n_slots < 1 || n_slots > 64 ||
      codes_capacity < MH_CODES_PAD)
    return MH_ERR_INVALID_ARG;
  const mh_dims &d = proto->dims;
  if (!d.width || !d.height || d.width > MH_MAX_DIM || d.height > MH_MAX_DIM ||
      d.block_width != (d.width + 7) / 8 || d.block_height != (d.height + 7) / 8)
    return MH_ERR_DIMS;
  *out = nullptr;
  mh_stream *s = new (std::nothrow) mh_stream();
  if (!s) return MH_ERR_CAPACITY;
  s->proto = *proto;
  s->proto.n_frames = 1;
  s->proto.d_frame_code_offsets = nullptr;
  s->cap = (codes_capacity + 15) & ~15ull;
  s->nb = (uint64_t)d.block_width * d.block_height;
  s->off_bytes = (s->nb * 4 + 15) & ~15ull;
  s->pitch = ((size_t)d.width + 7) & ~(size_t)7;
  s->out_bytes = s->pitch * d.height;
  s->slots.resize(n_slots);
  const bool want_init = proto->d_block_init != nullptr;
  // MH_STREAM_GRAPHS=0: direct launches instead of per-slot graph replays (A/B)
  const char *ge = std::getenv("MH_STREAM_GRAPHS");
  s->graphs = !(ge && ge[0] == '0');
  int rc = MH_OK;
  if (hipGetDevice(&s->device) != hipSuccess) rc = MH_ERR_HIP;
  for (uint32_t i = 0; i < n_slots && rc == MH_OK; ++i) {
    mh_stream::Slot &sl = s->slots[i];
    if (d_outputs) {
      sl.out = d_outputs[i];
      sl.own_out = false;
      if (!sl.out || ((uintptr_t)sl.out & 7u)) {
        rc = MH_ERR_ALIGN;
        break;
      }
    }
    if (hipMalloc(&sl.base, s->off_bytes + s->cap) != hipSuccess ||
        (want_init && hipMalloc(&sl.init, s->nb) != hipSuccess) ||
        (!d_outputs && hipMalloc(&sl.out, s->out_bytes) != hipSuccess) ||
        hipMemset(sl.base, 0, s->off_bytes + s->cap) != hipSuccess ||
        hipEventCreate(&sl.start) != hipSuccess || hipEventCreate(&sl.done) != hipSuccess ||
        hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking) != hipSuccess) {
      rc = MH_ERR_HIP;
      break;
    }
    sl.offsets = reinterpret_cast<uint32_t *>(sl.base);
    sl.codes = sl.base + s->off_bytes;
    if (want_init && hipMemset(sl.init, 0, s->nb) != hipSuccess) {
      rc = MH_ERR_HIP;
      break;
    }
    // The decode of this slot, captured once: the slot's buffers never move, and
    // codes_bytes = the slot capacity (the kernel bounds a frame's last block by
    // its 64 x 16-bit maximum, not by the buffer end).
    mh_frame f = s->proto;
    f.d_codes = sl.codes;
    f.codes_bytes = s->cap;
    f.d_block_offsets = sl.offsets;
    f.d_block_init = sl.init;
    // one eager decode first: validates the arguments and caches the launch
    // geometry queries outside the capture
    hipStream_t cs = sl.stream;
    const int wrc = mh_decode(&f, sl.out, s->pitch, s->out_bytes, cs);
    if (wrc != MH_OK) {
      rc = wrc;
      break;
    }
    if (!s->graphs) continue;
    if (hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal) != hipSuccess) {
      rc = MH_ERR_HIP;
      break;
    }
    const int drc = mh_decode(&f, sl.out, s->pitch, s->out_bytes, cs);
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(cs, &g);
    sl.graph = g;
    if (drc != MH_OK || e != hipSuccess) {
      rc = drc != MH_OK ? drc : MH_ERR_HIP;
      break;
    }
    if (hipGraphInstantiate(&sl.exec, sl.graph, nullptr, nullptr, 0) != hipSuccess) {
      rc = MH_ERR_HIP;
      break;
    }
  }
  if (rc == MH_OK && hipDeviceSynchronize() != hipSuccess) rc = MH_ERR_HIP;
  if (rc != MH_OK) {
    release(s);
    return rc;
  }
  *out = s;
  return MH_OK;
}

int mh_stream_submit(mh_stream *s, const uint8_t *h_codes, uint64_t codes_bytes,
                     const uint32_t *h_block_offsets, const uint8_t *h_block_init,
                     uint32_t *slot_out) {
  if (!s || !h_codes || !h_block_offsets) return MH_ERR_INVALID_ARG;
  if (codes_bytes < MH_CODES_PAD || codes_bytes > s->cap) return MH_ERR_CAPACITY;
  if (!h_block_init != !s->slots[0].init) return MH_ERR_INVALID_ARG;
  const uint32_t k = s->next;
  mh_stream::Slot &sl = s->slots[k];
  DeviceGuard dg(s->device);
  if (!dg.ok) return MH_ERR_HIP;
  if (hipEventRecord(sl.start, sl.stream) != hipSuccess) return MH_ERR_HIP;
  // copy then decode on the slot's own stream (its previous decode is ahead in it).
  // Host offsets and codes laid out like the slot ([offsets, padded to 16 B][codes]):
  // one DMA; otherwise two
  const bool packed = h_codes == reinterpret_cast<const uint8_t *>(h_block_offsets) + s->off_bytes;
  if ((packed ? hipMemcpyAsync(sl.base, h_block_offsets, s->off_bytes + codes_bytes,
                               hipMemcpyHostToDevice, sl.stream) != hipSuccess
              : (hipMemcpyAsync(sl.codes, h_codes, codes_bytes, hipMemcpyHostToDevice, sl.stream) !=
                     hipSuccess ||
                 hipMemcpyAsync(sl.offsets, h_block_offsets, s->nb * 4, hipMemcpyHostToDevice,
                                sl.stream) != hipSuccess)) ||
      (h_block_init &&
       hipMemcpyAsync(sl.init, h_block_init, s->nb, hipMemcpyHostToDevice, sl.stream) != hipSuccess) ||
      (s->graphs ? hipGraphLaunch(sl.exec, sl.stream) != hipSuccess : !decode_slot(s, sl, sl.stream)) ||
      hipEventRecord(sl.done, sl.stream) != hipSuccess)
    return MH_ERR_HIP;
  sl.used = true;
  s->last = k;
  s->next = (k + 1) % (uint32_t)s->slots.size();
  if (slot_out) *slot_out = k;
  return MH_OK;
}

uint8_t *mh_stream_output(mh_stream *s, uint32_t slot, size_t *out_pitch) {
  if (!s || slot >= s->slots.size()) return nullptr;
  if (out_pitch) *out_pitch = s->pitch;
  return s->slots[slot].out;
}

void *mh_stream_compute_stream(mh_stream *s) { return s ? (void *)s->slots[s->last].stream : nullptr; }

void *mh_stream_slot_stream(mh_stream *s, uint32_t slot) {
  return (s && slot < s->slots.size()) ? (void *)s->slots[slot].stream : nullptr;
}

int mh_stream_wait(mh_stream *s, uint32_t slot) {
  if (!s || slot >= s->slots.size()) return MH_ERR_INVALID_ARG;
  if (!s->slots[slot].used) return MH_OK;
  return hipEventSynchronize(s->slots[slot].done) == hipSuccess ? MH_OK : MH_ERR_HIP;
}

int mh_stream_slot_time(mh_stream *s, uint32_t slot, float *ms) {
  if (!s || slot >= s->slots.size() || !ms) return MH_ERR_INVALID_ARG;
  const mh_stream::Slot &sl = s->slots[slot];
  if (!sl.used) return MH_ERR_INVALID_ARG;
  if (hipEventSynchronize(sl.done) != hipSuccess) return MH_ERR_HIP;
  return hipEventElapsedTime(ms, sl.start, sl.done) == hipSuccess ? MH_OK : MH_ERR_HIP;
}

int mh_stream_device(mh_stream *s) { return s ? s->device : -1; }

int mh_stream_synchronize(mh_stream *s) {
  if (!s) return MH_ERR_INVALID_ARG;
  DeviceGuard dg(s->device);
  for (auto &sl : s->slots)
    if (sl.stream && hipStreamSynchronize(sl.stream) != hipSuccess) return MH_ERR_HIP;
  return MH_OK;
}

int mh_stream_destroy(mh_stream *s) {
  if (!s) return MH_ERR_INVALID_ARG;
  const int rc = mh_stream_synchronize(s);
  DeviceGuard dg(s->device);
  release(s);
  return rc;
}

// ---- stream groups: frames round-robined over several devices (config 5 on N
// GPUs). One mh_stream per member, each created on its device; a submit goes to
// the next member in turn with that member's device made current for the call.
struct mh_stream_group {
  std::vector<mh_stream *> members;
  uint32_t next = 0;
};

int mh_stream_group_create(const mh_frame *protos, uint32_t n_members, const int *devices,
                           uint64_t codes_capacity, uint32_t slots_per_member,
                           mh_stream_group **out) {
  if (!protos || !devices || !out || n_members < 1 || n_members > 64) return MH_ERR_INVALID_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) return MH_ERR_HIP;
  for (uint32_t i = 0; i < n_members; ++i)
    if (devices[i] < 0 || devices[i] >= ndev) return MH_ERR_INVALID_ARG;
  mh_stream_group *g = new (std::nothrow) mh_stream_group();
  if (!g) return MH_ERR_CAPACITY;
  int rc = MH_OK;
  for (uint32_t i = 0; i < n_members && rc == MH_OK; ++i) {
    DeviceGuard dg(devices[i]);
    if (!dg.ok) {
      rc = MH_ERR_HIP;
      break;
    }
    mh_stream *s = nullptr;
    rc = mh_stream_create(&protos[i], codes_capacity, slots_per_member, nullptr, &s);
    if (rc == MH_OK) g->members.push_back(s);
  }
  if (rc != MH_OK) {
    (void)mh_stream_group_destroy(g);
    return rc;
  }
  *out = g;
  return MH_OK;
}

int mh_stream_group_submit(mh_stream_group *g, const uint8_t *h_codes, uint64_t codes_bytes,
                           const uint32_t *h_block_offsets, const uint8_t *h_block_init,
                           uint32_t *member, uint32_t *slot) {
  if (!g || g->members.empty()) return MH_ERR_INVALID_ARG;
  const uint32_t m = g->next;
  const int rc = mh_stream_submit(g->members[m], h_codes, codes_bytes, h_block_offsets, h_block_init, slot);
  if (rc != MH_OK) return rc;
  g->next = (m + 1) % (uint32_t)g->members.size();
  if (member) *member = m;
  return MH_OK;
}

mh_stream *mh_stream_group_member(mh_stream_group *g, uint32_t member) {
  return (g && member < g->members.size()) ? g->members[member] : nullptr;
}

uint32_t mh_stream_group_size(const mh_stream_group *g) { return g ? (uint32_t)g->members.size() : 0u; }

int mh_stream_group_synchronize(mh_stream_group *g) {
  if (!g) return MH_ERR_INVALID_ARG;
  int rc = MH_OK;
  for (mh_stream *s : g->members) {
    const int r = mh_stream_synchronize(s);
    if (r != MH_OK) rc = r;
  }
  return rc;
}

int mh_stream_group_destroy(mh_stream_group *g) {
  if (!g) return MH_ERR_INVALID_ARG;
  int rc = MH_OK;
  for (mh_stream *s : g->members) {
    const int r = mh_stream_destroy(s);
    if (r != MH_OK) rc = r;
  }
  delete g;
  return rc;
}

}  // extern "C"

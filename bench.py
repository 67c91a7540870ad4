#!/usr/bin/env python3
"""bench.py -- decoded MB/s of 2048x1536 8-bit grayscale frames on MI355X.

BASELINE.json metric: "decoded MB/s (and Mpixels/s) at 2048x1536 grayscale,
1/2/4/8 GPU + CPU ref". MB = 1e6 bytes of decoded raster (1 byte per pixel, so
Mpixel/s is the same number).

A step is one pass of the hot path over one batch of input: by default
(--workload frame, BASELINE config 2) one kernel launch that decodes one
2048x1536 frame per GPU. Inputs are resident in HBM before timing starts: each
rank holds --frames (128) distinct block-shuffled BigBridge frames (the reference's
own TEST_IMAGE4 asset; every shuffle shares one canonical table).

Every clocked region is COLD, as every frame of the reference's renderer is new data
(Shared/AAPLRenderer.m:1178-1921): it decodes frames no earlier region touched (the
K eager launches of a region take the next K resident frames; the long launches --
the 64-frame batch, the 8192^2 frame -- cycle over >= 2 launches of >= 337 MB), and
a 1 GiB device copy evicts the 256 MiB Infinity Cache and the L2s right before the
region, off the clock. `warm_value` is a region that re-decodes the launches the region
before it decoded, without the flush: for the one-frame workload (20 frames, 106 MB)
those inputs are still in the Infinity Cache; for the long launches, which cycle over
>= 2 launch sets of >= 113 MB, they are not, so there warm ~ cold. Round 3's method (one
resident launch re-decoded: the 138 MB random frame entirely in the 256 MiB cache) runs
the same kernels 5-11 % faster (profiles/r05_bisect_ab.txt).
The K launches are enqueued behind a launch gate before the clock starts (short
launches eagerly, long ones as hipGraph replays). `roofline.kernel_us_avg` is the
timed region's own steady launch period from HIP events on the launch stream.

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): one process
per GPU; rank 0 broadcasts the 256-byte canonical header over RCCL (xGMI) once and every
rank builds T1/T2 and its decode table on its own GPU (mh_build_tables_device); frames
are sharded (each rank decodes its own), no collective on the data path;
value = all frames decoded / max-over-ranks wall time ("weak" scaling).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import json
import os
import socket
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "decoded MB/s (and Mpixels/s) at 2048×1536 grayscale, 1/2/4/8 GPU + CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", choices=["frame", "batch", "tile8192", "tile8192_random"], default="frame")
    ap.add_argument("--frames", type=int, default=128,
                    help="distinct resident frames per rank (>= 2 batch launches: cold regions)")
    ap.add_argument("--batch", type=int, default=64, help="frames per launch for --workload batch")
    ap.add_argument("--no-extras", action="store_true", help="skip the batch/tile side measurements")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (default: the affinity set, capped by the cgroup quota)")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of a hipGraph")
    ap.add_argument("--dist", action="store_true",
                    help="take the multi-GPU path (process group, table broadcast, all-ranks extras) even "
                         "at world size 1: RCCL exercised on a one-GPU box")
    return ap.parse_args(argv)


# --------------------------------------------------------------------------------------
def encode_many(imgs, threads=8):
    import metalhuffman_amd as mh
    with cf.ThreadPoolExecutor(threads) as ex:  # ctypes releases the GIL
        return list(ex.map(mh.encode_frame, imgs))


def algo_bytes(efs, t2_bytes: int) -> int:
    """Algorithmic HBM bytes of one launch: payload codes +
    block offsets + decoded raster per frame, T1 + T2 once per launch."""
    per = sum(ef.payload_bytes + 4 * ef.n_blocks + ef.width * ef.height for ef in efs)
    return per + 512 + t2_bytes


def algo_read_bytes(efs, t2_bytes: int) -> int:
    """The read share of algo_bytes (codes + offsets + tables): what north_star's
    "HBM read roofline" fraction is computed from."""
    return sum(ef.payload_bytes + 4 * ef.n_blocks for ef in efs) + 512 + t2_bytes


# A/B switch for decode-only flags (e.g. 2 = MH_FLAG_LANE_PAIRS, scripts/gpu_lane_pairs_ab.sh);
# the parity guard (Workload.verify) decodes through the same flags before anything is timed
DECODE_FLAGS = int(os.environ.get("MH_BENCH_DECODE_FLAGS", "0"), 0)
# Inside an eager timed region every launch after the first goes out with
# MH_FLAG_ANY_ORDER (no barrier bit; each launch writes its own raster). The first launch
# keeps the barrier, so nothing starts before the region opens. On gfx950 the dispatches
# do not overlap (scripts/micro/any_order_probe.hip); the gap between them shrinks: 5.56-5.62
# vs 5.78-5.82 us per launch over 20/64-launch regions (profiles/r02_v19_any_order_ab.txt).
MH_FLAG_ANY_ORDER = 0x4
FLUSH_BYTES = 512 << 20  # x2 buffers: 1 GiB of HBM traffic, 4x the 256 MiB Infinity Cache


class _Flush:
    """Evicts the Infinity Cache (MALL, 256 MiB) and the XCD L2s before a cold timed
    region: one device copy of 512 MiB (512 MiB read + 512 MiB written), issued on the
    launch stream before the region's opening synchronize, so it is off the clock. (A
    read-only eviction -- a reduction over 1 GiB, nothing left dirty -- left the batch
    and 8192^2 launches 7-10 % slower: profiles/r05_flush_method_ab.txt.)"""

    def __init__(self):
        self.bufs = {}

    def __call__(self, dev):
        if dev not in self.bufs:
            a = torch.empty(FLUSH_BYTES, dtype=torch.uint8, device=dev)
            a.fill_(1)
            self.bufs[dev] = (a, torch.empty_like(a))
        a, b = self.bufs[dev]
        b.copy_(a)


FLUSH = _Flush()


class Workload:
    """A set of launches (one DeviceFrames each) cycled over by the steps."""

    def __init__(self, name, launches, tables, pixels_per_launch, bytes_per_launch, device, refs=None,
                 read_bytes=None):
        from metalhuffman_amd import decoder as D
        self.D = D
        self.name = name
        self.launches = launches
        self.refs = refs  # per launch: the frames' input rasters as u8[n, H, W] (device), or None
        self.tables = tables
        self.pixels = pixels_per_launch
        self.bytes = bytes_per_launch
        self.read_bytes = read_bytes
        self.ungated_wall = None
        self.warm_wall = None
        self.device = device
        self.base = 0  # eager regions decode launches base, base+1, ... (advanced per cold region)
        self.outs = [torch.empty((f.n_frames, f.height, (f.width + 7) // 8 * 8), dtype=torch.uint8,
                                 device=device) for f in launches]

    def launch(self, i, stream=None, relaxed=False):
        j = (self.base + i) % len(self.launches)
        self.D.decode(self.launches[j], self.tables, self.outs[j], stream=stream,
                      extra_flags=DECODE_FLAGS | (MH_FLAG_ANY_ORDER if relaxed else 0))

    def run_streams(self, steps, nstreams, reps=3):
        """The same one-frame launches round-robined over `nstreams` HIP streams: launch
        i goes to stream i % nstreams (each launch still decodes one frame into its own
        buffer), all queued behind one launch gate per stream, opened together; the
        clock runs from the gate's opening to the closing synchronize. Independent
        frames overlap on the device (one frame fills <= one wave per SIMD). Each region
        decodes frames no earlier region touched, after the cache flush (cold inputs).
        Best of `reps` regions -> seconds per launch."""
        dev = self.device
        if not GATE.ok():
            return None
        assert len(self.launches) % nstreams == 0  # launch j stays on one stream
        streams = [torch.cuda.Stream(dev) for _ in range(nstreams)]
        best = None
        for _ in range(reps + 1):  # the first region warms the streams
            self.base = (self.base + steps) % len(self.launches)
            self.base -= self.base % nstreams
            FLUSH(dev)
            torch.cuda.synchronize(dev)
            for st in streams:
                GATE.arm(st.cuda_stream)
            for i in range(steps):
                self.launch(i, stream=streams[i % nstreams])
            t0 = time.perf_counter()
            GATE.open()
            torch.cuda.synchronize(dev)
            w = time.perf_counter() - t0
            best = w if best is None or w < best else best
        return best / steps

    def verify(self) -> int:
        """Parity guard before any timing: every resident launch is decoded once and
        EVERY frame of it compared with its encoder input on the device (the DEBUG
        self-check of Shared/AAPLRenderer.m:616-650). Returns the frames checked;
        raises on the first mismatch. No switch turns it off."""
        if self.refs is None:
            raise RuntimeError(f"{self.name}: no reference frames to verify against")
        n = 0
        base, self.base = self.base, 0
        for j, fr in enumerate(self.launches):
            self.launch(j)
            torch.cuda.synchronize(self.device)
            got = self.outs[j][..., : fr.width]
            for i in range(fr.n_frames):
                if not torch.equal(got[i], self.refs[j][i]):
                    raise SystemExit(f"bench: {self.name} launch {j} frame {i} differs from the encoder input")
                n += 1
        self.base = base
        return n

    def check_outputs(self) -> None:
        """After the timed regions: every launch's raster (as the any-order and rotated
        regions left it) still equals its encoder input."""
        for j, fr in enumerate(self.launches):
            if not torch.equal(self.outs[j][..., : fr.width], self.refs[j]):
                raise SystemExit(f"bench: {self.name} launch {j} differs from the encoder input after timing")

    def run(self, steps, warmup, use_graph=True, world=1, settle_ms=50.0):
        """Timed regions of `steps` launches each, bracketed by barrier + synchronize;
        wall = max over ranks. Every clocked region is COLD: the launches it decodes were
        not touched by the region before it (eager regions advance `base` by `steps`;
        graph regions cycle over >= 2 launches of >= 337 MB each) and a 1 GiB copy evicts
        the 256 MiB Infinity Cache and the L2s right before it (off the clock), as every
        frame of the reference's renderer is new data (Shared/AAPLRenderer.m:1178-1921).
        The previous warm method (the region re-decodes the frames the region before it
        just decoded) is reported as `warm_wall`.
        -> (wall_s, gpu_region_ms, per-launch kernel ms list)."""
        dev = self.device
        for i in range(warmup):
            self.launch(i)
        torch.cuda.synchronize(dev)
        # Long launches (>= LONG_LAUNCH_PIXELS decoded per launch: the 64-frame batch, the
        # 8192^2 frame; 20-70 us each) replay a graph of LONG_GRAPH_LAUNCHES launches
        # K / LONG_GRAPH_LAUNCHES times; the first replay is queued behind the launch gate,
        # the rest are enqueued once it opens (the host runs ~1 ms ahead of the GPU).
        # Queuing every replay behind the gate times the same unprofiled (66.9-67.0 vs
        # 66.9-67.6 us per batch launch) but ran 15-20 % slower per dispatch under
        # rocprofv3 (78.3 vs 68.3 us batch, 30.4 vs 25.3 us 8192^2), which made the profile
        # disagree with the line (profiles/r03_window_ab.txt, r03_gate_rocprof_artifact.txt);
        # plain eager regions dispatch 5-8 % slower than queued ones
        # (profiles/r03_long_launch_ab.txt). Short launches (one 2048x1536 frame, ~5.5 us)
        # go out eagerly behind the gate. Decided by size, not by a timing probe: under a
        # profiler the probe itself slows.
        self.long_launches = self.pixels >= LONG_LAUNCH_PIXELS
        window = self.long_launches
        G = steps  # launches per captured graph
        if self.long_launches and steps % LONG_GRAPH_LAUNCHES == 0:
            G = LONG_GRAPH_LAUNCHES
        self.graph_launches = G
        graph = None

        def replay_all():  # the K launches: K / G replays of the G-launch graph
            for _ in range(steps // G):
                graph.replay()
        if use_graph:
            try:
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    for i in range(G):
                        self.launch(i)
                graph.replay()  # first replay off the clock (instantiation effects)
                torch.cuda.synchronize(dev)
                # untimed replays for ~settle_ms right before the timed one: the timed
                # replay starts on a busy, clocked-up GPU (a single cold replay of a
                # 20-step graph measured 30-50 % slower than the median of many)
                t_end = time.perf_counter() + settle_ms * 1e-3
                while time.perf_counter() < t_end:
                    replay_all()
                    torch.cuda.synchronize(dev)
            except Exception as e:  # pragma: no cover - fall back to eager launches
                print(f"[bench] hipGraph capture failed ({e}); eager launches", file=sys.stderr)
                graph = None
        # the process's first timing-event records initialise HIP's event timing
        # (measured +40 us on the first timed region): do that off the clock
        for _ in range(2):
            wa, wb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            wa.record()
            if graph is not None:
                replay_all()
            wb.record()
            torch.cuda.synchronize(dev)
            wa.elapsed_time(wb)
        # eager behind the gate for short regions: there a replayed graph's ~6 us start
        # costs most (profiles/r02_v10_gated_eager_vs_graph_ab.txt); long regions replay
        eager_gated = steps <= 64 and not self.long_launches
        G_unit = G if (graph is not None and not eager_gated) else 1

        def timed(gated=True, events=True, mark=False, cold=True):
            """One timed region of exactly `steps` launches. Gated: the launches are
            enqueued behind the launch gate (scripts/micro/launch_gate.hip) after the
            opening synchronize, and the clock starts when the host opens it -- every
            decode runs inside the region, the host's enqueue latency does not.
            cold: decode the next `steps` launches (eager) after the cache flush;
            otherwise the same launches as the previous region, no flush (warm)."""
            r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            rA = torch.cuda.Event(enable_timing=True)  # after the region's first launch (or replay)
            unit = G_unit if gated else (G if graph is not None else 1)
            if dist.is_initialized():
                dist.barrier()
            st = torch.cuda.current_stream(dev).cuda_stream
            if cold:
                if eager_gated or graph is None:
                    self.base = (self.base + steps) % len(self.launches)
                FLUSH(dev)
            if mark and GATE.ok():
                GATE.marker(st, 1)  # before the gate / the first launch: off the clock
            torch.cuda.synchronize(dev)
            if gated:
                GATE.arm(torch.cuda.current_stream(dev).cuda_stream)
            nrep = steps // G
            # replays queued behind the gate (window mode: the first only, the rest are
            # enqueued once the gate is open, the host running ahead of the GPU)
            pre = nrep if not (gated and window) else min(1, nrep)
            if gated:
                if events:
                    r0.record()
                if graph is not None and not eager_gated:
                    for r in range(pre):
                        graph.replay()
                        if r == 0 and events:
                            rA.record()
                else:
                    # any-order only when every launch of the region writes its own raster
                    # (no launch may overlap one that writes the same buffer)
                    relax = len(self.launches) >= steps
                    for i in range(steps):
                        self.launch(i, relaxed=relax and i > 0)
                        if i == 0 and events:
                            rA.record()
                if events and pre == nrep:
                    r1.record()
            # (no barrier while a gate is armed: an RCCL barrier would queue behind it;
            # each rank times its own region, the max over ranks is taken below)
            t0 = time.perf_counter()
            if gated:
                GATE.open()
                if pre < nrep:
                    for r in range(pre, nrep):
                        graph.replay()
                    if events:
                        r1.record()
            else:
                r0.record()
                if graph is not None:
                    for r in range(steps // G):
                        graph.replay()
                        if r == 0:
                            rA.record()
                else:
                    for i in range(steps):
                        self.launch(i)
                        if i == 0:
                            rA.record()
                r1.record()
            if mark and GATE.ok():
                GATE.marker(st, 2)  # after the last launch (one empty kernel inside a plain region's wall)
            torch.cuda.synchronize(dev)
            w = time.perf_counter() - t0
            if dist.is_initialized():
                dist.barrier()
                on = dev if dist.get_backend() == "nccl" else torch.device("cpu")
                t = torch.tensor([w], dtype=torch.float64, device=on)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                w = float(t.item())
            # steady-state launch time: the launches after the first unit (the first one also
            # holds the gate's release and the first dispatch's start-up)
            steady = (rA.elapsed_time(r1) / (steps - unit) if events and steps > unit else
                      (r0.elapsed_time(r1) / steps if events else None))
            return w, (r0.elapsed_time(r1) if events else None), (steady, unit)

        if GATE.ok():
            timed(events=False, cold=False)  # the gate's own first launch off the clock
            # warm (reported beside): the same launches again, no flush
            self.warm_wall, _, _ = timed(events=False, cold=False)
            # The clocked region holds only the K launches: its two HIP event records
            # (markers in the queue) cost ~7 us per region at 20 steps (510 vs 482 x10^3
            # MB/s interleaved, profiles/r02_v13_region_events_ab.txt), so the event-timed
            # region is a second, identical (cold) one.
            wall, _, _ = timed(events=False)
            _, region_ms, (steady_ms, self.steady_unit) = timed(mark=True)
            self.ungated_wall, _, _ = timed(gated=False)
            self.timed_launch = (("eager behind the launch gate, launches 2..K with MH_FLAG_ANY_ORDER")
                                 if eager_gated else
                                 f"{steps // G} replays of a {G}-launch hipGraph, the first behind the launch gate, "
                                 "the rest enqueued once it opens")
        else:
            wall, region_ms, (steady_ms, self.steady_unit) = timed(gated=False, mark=True)
            self.ungated_wall = None
            self.timed_launch = "hipGraph" if graph is not None else "eager"
        self.timed_launch += "; cold inputs (launches no earlier region touched, 1 GiB cache flush before each region)"
        self.region_kernel_ms = region_ms / steps
        self.steady_kernel_ms = steady_ms
        # Per-launch kernel duration of the same launches replayed as graphs back to back
        # (>= 200 launches, warm) between one event pair: informational.
        if graph is not None and G < steps:
            ka, kb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(dev)
            ka.record()
            replay_all()
            kb.record()
            torch.cuda.synchronize(dev)
            self.kernel_ms = ka.elapsed_time(kb) / steps
        elif graph is not None:
            # one graph of >= 200 launches (a replayed graph's first kernel starts ~6 us
            # late: 10 replays of a 20-launch graph would add ~0.3 us per launch)
            kg, nk = graph, steps
            if steps < 200:
                nk = 200
                kg = torch.cuda.CUDAGraph()
                with torch.cuda.graph(kg):
                    for i in range(nk):
                        self.launch(i)
                kg.replay()
            ka, kb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(dev)
            ka.record()
            kg.replay()
            kb.record()
            torch.cuda.synchronize(dev)
            self.kernel_ms = ka.elapsed_time(kb) / nk
            del kg
        else:
            self.kernel_ms = None
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(steps)]
        for i in range(steps):
            ev[i][0].record()
            self.launch(i)
            ev[i][1].record()
        torch.cuda.synchronize(dev)
        kms = [a.elapsed_time(b) for a, b in ev]
        return wall, region_ms, kms


TRAFFIC_JSON = os.path.join(ROOT, "profiles", "traffic.json")
TILE_FRAMES = 6  # distinct 8192^2 frames per tile workload
LONG_LAUNCH_PIXELS = 16 << 20  # Workload.run: launches decoding this many pixels are "long"
LONG_GRAPH_LAUNCHES = 16       # ... and replay a graph of this many launches K / 16 times


def measured_traffic(workload: str):
    """HBM bytes per launch of this workload from the committed PMC profile
    (scripts/gpu_traffic.sh: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, FETCH x2 on
    gfx950), or None when no profile covers it."""
    try:
        with open(TRAFFIC_JSON) as f:
            rec = json.load(f)["per_launch_median"].get(workload)
        return int(rec["traffic_bytes"]) if rec else None
    except (OSError, KeyError, ValueError):
        return None


ACHIEVABLE = {}  # filled from hbm_probe() before the roofline lines (rank 0, N=1)


class _Gate:
    """The timed-region launch gate (scripts/micro/liblaunch_gate.so): a one-wave
    kernel polling a host-mapped flag, so the K launches can be enqueued before the
    clock starts."""

    def __init__(self):
        self.lib = None
        self.h = self.d = None

    def ok(self) -> bool:
        if self.lib is None:
            import ctypes
            path = os.path.join(ROOT, "scripts", "micro", "liblaunch_gate.so")
            if not os.path.exists(path):
                return False
            lib = ctypes.CDLL(path)
            lib.gate_create.argtypes = [ctypes.POINTER(ctypes.c_void_p)] * 2
            lib.gate_arm.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
            lib.gate_open.argtypes = [ctypes.c_void_p]
            lib.trace_marker.argtypes = [ctypes.c_void_p, ctypes.c_uint]
            h, d = ctypes.c_void_p(), ctypes.c_void_p()
            if lib.gate_create(ctypes.byref(h), ctypes.byref(d)) != 0:
                return False
            self.lib, self.h, self.d = lib, h, d
        return True

    def arm(self, stream: int) -> None:
        if self.lib.gate_arm(self.h, self.d, stream, 200_000) != 0:  # opens by itself after 200 ms
            raise RuntimeError("launch gate: kernel launch failed")

    def marker(self, stream: int, tag: int) -> None:
        """An empty kernel on `stream`: brackets the events-timed region in a rocprofv3
        trace (scripts/ktrace_summary.py)."""
        if self.lib is not None and self.lib.trace_marker(stream, tag) != 0:
            raise RuntimeError("trace marker: kernel launch failed")

    def open(self) -> None:
        self.lib.gate_open(self.h)


GATE = _Gate()
def roofline(bytes_per_launch, region_ms, steps, eager_ms=None, workload=None, read_bytes=None,
             kernel_ms=None, steady_ms=None, steady_unit=1):
    """achieved = algorithmic bytes of one launch / the launch's average duration,
    the latter from the timed region itself, by HIP events on the launch stream:
    kernel_us_avg = (end of the region - end of its first launch or first graph replay of
    `steady_unit` launches) / (K - steady_unit), i.e. the back-to-back launch period inside
    the region without the gate's release and the first dispatch's start-up (which
    region_us_per_launch = the whole region / K still holds). rocprofv3 --kernel-trace of
    the same command gives the same quantity from its dispatch timestamps
    (scripts/ktrace_summary.py `timed_steady`; profiles/r03_ktrace_summary.txt).
    graph_us_per_launch: the same launches replayed as graphs (Workload.run), for reference.
    frac is against the 8 TB/s spec; frac_of_achievable against a plain streaming
    kernel with the decoder's read:write mix measured on the same box."""
    avg_s = (steady_ms if steady_ms else region_ms / steps) * 1e-3
    ach = bytes_per_launch / avg_s / 1e9
    r = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(ach / HBM_PEAK_GBS, 4),
         "traffic": measured_traffic(workload) if workload else None,
         "kernel_us_avg": round(avg_s * 1e6, 3),
         "kernel_us_source": (f"HIP events over the timed region after its first {steady_unit} launch(es), "
                              f"/ (K - {steady_unit})" if steady_ms else "HIP events around the timed region / K"),
         "kernel_us_steady_unit": steady_unit if steady_ms else 0,
         "region_us_per_launch": round(region_ms * 1e3 / steps, 3),
         "graph_us_per_launch": round(kernel_ms * 1e3, 3) if kernel_ms else None,
         "algorithmic_bytes_per_launch": int(bytes_per_launch)}
    mix = ACHIEVABLE.get("mix_2r3w_GBps")
    if mix:
        r["achievable_mix_GBps"] = mix
        r["frac_of_achievable"] = round(ach / mix, 4)
    if read_bytes:
        # north_star's "per-GPU HBM read roofline": the launch's read bytes (codes,
        # offsets, tables) over its duration, against the spec and the measured
        # read-only stream
        rd = read_bytes / avg_s / 1e9
        r["read_bytes_per_launch"] = int(read_bytes)
        r["read_achieved"] = round(rd, 1)
        r["read_frac"] = round(rd / HBM_PEAK_GBS, 4)
        if ACHIEVABLE.get("read_GBps"):
            r["read_frac_of_achievable"] = round(rd / ACHIEVABLE["read_GBps"], 4)
    if eager_ms:
        # one launch at a time with an event pair each (includes launch latency)
        r["eager_launch_us_median"] = round(float(np.median(eager_ms)) * 1e3, 3)
    return r


def stream_h2d(efs, tables, device, n_frames=2048, n_cold=1000, n_paced=1000, sync=None):
    """BASELINE config 5 on this rank's GPU through the native stream group
    (mh_stream_group_*, one member here; N members round-robin frames over N GPUs):
    frames start in pinned host memory; each is copied H2D (codes + block offsets, one
    DMA) into one of two device slots and decoded by that slot's captured graph, both
    on the slot's own stream, so the copy of frame i+1 overlaps the decode of frame i.
    Reports, on a freshly created stream (no warm-up excluded): the first n_cold
    frames back to back and the very first frame's latency; then the sustained rate;
    then n_paced frames one at a time (a 30 FPS consumer: nothing queued) with host
    latency submit -> decoded (p50/p99/max) and device latency H2D start -> decode end.
    Never the headline `value` (inputs are not resident in HBM)."""
    from metalhuffman_amd.stream import FrameStreamGroup, pinned_frame
    W, H = efs[0].width, efs[0].height
    hosts = [pinned_frame(ef) for ef in efs]
    cap = max(ef.codes.size for ef in efs)
    g = FrameStreamGroup([tables], W, H, cap, slots=2)
    c, o = hosts[0]
    t = time.perf_counter()
    m, sl = g.submit(c, o)
    g.wait(m, sl)
    first_us = (time.perf_counter() - t) * 1e6

    def run(count, start=0):
        for i in range(count):
            c, o = hosts[(start + i) % len(hosts)]
            g.submit(c, o)
        g.synchronize()

    t0 = time.perf_counter()
    run(n_cold, 1)
    cold_wall = time.perf_counter() - t0
    if sync is not None:  # multi-rank: every rank's sustained phase starts together
        sync()
    t0 = time.perf_counter()
    run(n_frames)
    wall = time.perf_counter() - t0
    host_lat, dev_lat = [], []
    last = None
    for i in range(n_paced):  # one frame in flight at a time
        c, o = hosts[i % len(hosts)]
        t = time.perf_counter()
        m, sl = g.submit(c, o)
        g.wait(m, sl)
        host_lat.append((time.perf_counter() - t) * 1e6)
        dev_lat.append(g.slot_time_ms(m, sl) * 1e3)
        last = (i % len(hosts), m, sl)
    out_last = g.output(last[1], last[2])[:, :W].clone()
    g.close()
    from metalhuffman_amd import decoder as D
    ref = D.decode(D.DeviceFrames.pack([efs[last[0]]], device), tables)
    torch.cuda.synchronize(device)
    if not torch.equal(ref[0, :, :W], out_last):
        raise SystemExit("bench: streamed frame differs from the resident decode")
    h2d = float(np.mean([ef.codes.size + 4 * ef.n_blocks for ef in efs]))
    pct = lambda v, q: round(float(np.percentile(v, q)), 1)
    return {"frames": n_frames, "fps": round(n_frames / wall, 1),
            "value_MBps_incl_pcie": round(n_frames * W * H / wall / 1e6, 1),
            "h2d_bytes_per_frame": int(h2d), "h2d_GBps": round(n_frames * h2d / wall / 1e9, 2),
            "cold_first_frames": n_cold + 1, "cold_fps": round(n_cold / cold_wall, 1),
            "cold_first_frame_latency_us": round(first_us, 1),
            "paced_frames": n_paced,
            "latency_us_p50": pct(host_lat, 50), "latency_us_p99": pct(host_lat, 99),
            "latency_us_max": round(max(host_lat), 1),
            "device_latency_us_p50": pct(dev_lat, 50), "device_latency_us_p99": pct(dev_lat, 99),
            "device_latency_us_max": round(max(dev_lat), 1),
            "slots": 2, "members": g.size,
            "launch": "native mh_stream_group: per slot one stream, one H2D DMA + a captured hipGraph decode per frame"}


def copy_bandwidth(device, nbytes=1 << 30, reps=20):
    """Achievable HBM bandwidth on this box: a device-to-device copy of 1 GiB
    (read + write bytes / time, best of `reps`), reported beside the spec peak
    (SURVEY.md 8(d))."""
    a = torch.empty(nbytes, dtype=torch.uint8, device=device)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize(device)
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b.copy_(a)
        e1.record()
        torch.cuda.synchronize(device)
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    del a, b
    return {"bytes_moved": 2 * nbytes, "best_ms": round(best, 4),
            "GBps": round(2 * nbytes / (best * 1e-3) / 1e9, 1), "kernel": "torch copy_ (D2D)"}


def hbm_probe(nbytes=1 << 30, reps=10):
    """Achievable HBM bandwidth on this box from scripts/micro/libhbm_probe.so (16-B
    vector streams, every CU busy): copy, read-only, write-only and the decoder's
    read:write mix (2:3), with non-temporal stores (as the decoder) and with
    default-policy stores. None when the probe was not built."""
    import ctypes
    path = os.path.join(ROOT, "scripts", "micro", "libhbm_probe.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.hbm_probe.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    out = {}
    for mode, name in ((0, "copy"), (1, "read"), (2, "write"), (3, "mix_2r3w"), (4, "copy_plainstore"),
                       (5, "write_plainstore"), (6, "mix_2r3w_plainstore")):
        g = ctypes.c_double()
        rc = lib.hbm_probe(mode, nbytes, reps, ctypes.byref(g))
        out[name + "_GBps"] = round(g.value, 1) if rc == 0 else None
    out["bytes_per_run"] = nbytes
    return out


def encode_rate(device, bb, reps=32):
    """The producer side: GPU encoder, synchronous (mh_encode_frame_device: one host
    sync per frame for the header and byte count) and device-only
    (mh_encode_frame_device_async: the Huffman tree on the device, frames enqueued
    back to back on one stream, then two frames in flight on two streams), vs the
    host codec (mh_encode_frame, one thread), all on
    BigBridge-shuffled frames, wall clock per frame."""
    import metalhuffman_amd as mh
    from metalhuffman_amd import frames as F
    from metalhuffman_amd.encoder import Encoder
    imgs = [F.block_shuffle(bb, 900 + k) for k in range(4)]
    dimgs = [torch.from_numpy(im).to(device) for im in imgs]
    enc = Encoder(bb.shape[1], bb.shape[0], device)
    codes = [torch.empty(enc.cap, dtype=torch.uint8, device=device) for _ in range(4)]
    for k in range(4):
        enc.encode(dimgs[k])
        enc.encode_async(dimgs[k], codes=codes[k])
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for k in range(reps):
        enc.encode(dimgs[k % 4])
    torch.cuda.synchronize(device)
    gpu_s = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for k in range(reps):
        enc.encode_async(dimgs[k % 4], codes=codes[k % 4])
    torch.cuda.synchronize(device)
    async_s = (time.perf_counter() - t0) / reps
    # frames in flight: one encoder (workspace) and one stream per slot, so one
    # frame's single-workgroup tree build overlaps the other's wide kernels
    def in_flight(nsl):
        encs = [Encoder(bb.shape[1], bb.shape[0], device) for _ in range(nsl)]
        streams = [torch.cuda.Stream(device) for _ in range(nsl)]
        cb = [torch.empty(enc.cap, dtype=torch.uint8, device=device) for _ in range(nsl)]
        for st in streams:
            st.wait_stream(torch.cuda.current_stream(device))
        for k in range(2 * nsl):
            encs[k % nsl].encode_async(dimgs[k % 4], stream=streams[k % nsl], codes=cb[k % nsl])
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for k in range(reps):
            encs[k % nsl].encode_async(dimgs[k % 4], stream=streams[k % nsl], codes=cb[k % nsl])
        torch.cuda.synchronize(device)
        return (time.perf_counter() - t0) / reps
    pipe_s = in_flight(2)
    pipe4_s = in_flight(4)
    # batched: 64 frames per call (mh_encode_frames_device_async, three launches),
    # each frame its own tree; calls back to back on one stream, after a warm-up call
    from metalhuffman_amd.encoder import BatchEncoder
    nbatch = 64
    benc = BatchEncoder(bb.shape[1], bb.shape[0], nbatch, device)
    bimgs = torch.from_numpy(np.stack([F.block_shuffle(bb, 950 + k) for k in range(nbatch)])).to(device)
    a = benc.encode_async(bimgs)
    torch.cuda.synchronize(device)
    if int((a.status != 0).sum().item()):
        raise SystemExit("bench: batched encode rejected a frame")
    for f in (0, nbatch - 1):  # parity guard: the host codec's bytes
        ref = mh.encode_frame(bimgs[f].cpu().numpy())
        if not np.array_equal(a.frame(f).codes.cpu().numpy(), ref.codes):
            raise SystemExit("bench: batched encode differs from the host codec")
    breps = 8
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(breps):
        benc.encode_async(bimgs)
    e1.record()
    torch.cuda.synchronize(device)
    batch_s = e0.elapsed_time(e1) * 1e-3 / (breps * nbatch)
    t0 = time.perf_counter()
    for k in range(4):
        mh.encode_frame(imgs[k])
    cpu_s = (time.perf_counter() - t0) / 4
    # algorithmic bytes of one encode: pixels in, code bytes + block offsets out (the
    # block-symbol intermediate is not counted: it is the encoder's own choice)
    ref = mh.encode_frame(imgs[0])
    alg = bb.size + ref.codes.size + 4 * ref.n_blocks
    return {"gpu_ms_per_frame": round(gpu_s * 1e3, 3), "gpu_MBps": round(bb.size / gpu_s / 1e6, 1),
            "algorithmic_bytes_per_frame": int(alg),
            "gpu_async_2streams_algorithmic_GBps": round(alg / pipe_s / 1e9, 1),
            "gpu_async_2streams_frac_of_8TBps": round(alg / pipe_s / 8e12, 4),
            "gpu_async_ms_per_frame": round(async_s * 1e3, 3),
            "gpu_async_MBps": round(bb.size / async_s / 1e6, 1),
            "gpu_async_2streams_ms_per_frame": round(pipe_s * 1e3, 3),
            "gpu_async_2streams_MBps": round(bb.size / pipe_s / 1e6, 1),
            "gpu_async_4streams_ms_per_frame": round(pipe4_s * 1e3, 3),
            "gpu_batch64_ms_per_frame": round(batch_s * 1e3, 4),
            "gpu_batch64_MBps": round(bb.size / batch_s / 1e6, 1),
            "gpu_batch64_algorithmic_GBps": round(alg / batch_s / 1e9, 1),
            "gpu_batch64_frac_of_8TBps": round(alg / batch_s / 8e12, 4),
            "gpu_batch64_method": (f"{breps} calls of {nbatch} block-shuffled BigBridge frames back to back on one "
                                   "stream (mh_encode_frames_device_async), HIP events, / frames"),
            "host_1thread_ms_per_frame": round(cpu_s * 1e3, 2), "host_1thread_MBps": round(bb.size / cpu_s / 1e6, 1)}


def cpu_share():
    """(threads this process may run on, the cgroup CPU quota in CPUs or None)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    return aff, quota


# port / reference speed on one core (profiles/r06_cpu_calibration.txt)
CPU_CALIBRATION_RATIO = 0.97
CPU_CALIBRATION_RANGE = (0.85, 1.23)


def cpu_baseline(efs, threads=None, target_s=2.0):
    """The reference's CPU decode (HuffmanUtil::decodeHuffmanBitsFromTables,
    Shared/HuffmanUtil.cpp:830-1046) restated in oracle/ (kind 'port': the reference's
    HuffmanUtil.cpp needs Apple's <simd/simd.h> and is unbuildable here; the port keeps
    its per-symbol 3-byte window reads and T1/T2 lookups). Calibration: SURVEY.md section 6
    timed the reference binary at 105.7 MB/s (BigBridge, one thread) in the build
    container; the port, timed the same way there (scripts/calibrate_cpu_baseline.py),
    ran at 0.85-1.23x that across sessions (profiles/r06_cpu_calibration.txt) -- carried
    as calibration_ratio (port / reference), so value / ratio estimates the reference.
    Timed on this host, frame-parallel:
      * one thread;
      * every CPU this process may use: the affinity set, capped by the cgroup CPU
        quota when one is set (`value`, `cores`), and the whole affinity set when
        the quota is smaller;
      * the full CPU pipeline decode + undelta + raster (1 thread and all CPUs).
    Each multi-thread sample is sized to ~target_s seconds from the 1-thread rate."""
    from oracle import oracle as O
    O.build()
    aff, quota = cpu_share()
    share = threads or (min(aff, max(1, int(quota))) if quota else aff)
    t1, t2 = efs[0].tables()
    W, H = efs[0].width, efs[0].height
    nsym = efs[0].n_blocks * 64
    px = W * H
    bufs = [ef.codes for ef in efs]
    one = O.time_decode_frames(t1, t2, nsym, bufs[:1], 1, reps=16)
    mb1 = 16 * px / one / 1e6

    def parallel(n_threads, fn):
        frames = max(len(bufs), n_threads)
        fb = [bufs[i % len(bufs)] for i in range(frames)]
        reps = max(1, int(round(target_s * mb1 * 1e6 * n_threads / (frames * px))))
        sec = fn(fb, n_threads, reps)
        return reps * frames * px / sec / 1e6, reps, frames, sec

    dec = lambda fb, n, r: O.time_decode_frames(t1, t2, nsym, fb, n, reps=r)
    pipe = lambda fb, n, r: O.time_decode_pipeline(t1, t2, W, H, fb, n, reps=r)
    mbn, reps, frames, sec = parallel(share, dec)
    p1 = O.time_decode_pipeline(t1, t2, W, H, bufs[:1], 1, reps=16)
    pn = parallel(share, pipe)
    out = {"value": round(mbn, 1), "unit": "MB/s", "cores": share, "kind": "port",
           "sample": f"{reps}x{frames} BigBridge-shuffle frames (2048x1536, 4.89 bit/sym), "
                     f"frame-parallel on {share} threads, {sec:.2f}s; oracle restatement of "
                     f"HuffmanUtil.cpp:830-1046 (gcc -O2); the reference's own decoder is "
                     f"unbuildable here, calibrated against its SURVEY 6 timing",
           "calibration_ratio": CPU_CALIBRATION_RATIO, "calibration_range": list(CPU_CALIBRATION_RANGE),
           "calibration_source": "profiles/r06_cpu_calibration.txt: port MB/s / the reference binary's "
                                 "105.7 MB/s (SURVEY.md 6), same container, one thread, BigBridge",
           "reference_equivalent_value": round(mbn / CPU_CALIBRATION_RATIO, 1),
           "single_thread_MBps": round(mb1, 1),
           "pipeline_decode_undelta_raster_1thread_MBps": round(16 * px / p1 / 1e6, 1),
           "pipeline_decode_undelta_raster_MBps": round(pn[0], 1),
           "affinity_threads": aff, "cgroup_cpu_quota": quota,
           "cpu_model": _cpu_model(), "host_nproc": os.cpu_count()}
    if aff > share:
        out["all_affinity_threads_MBps"] = round(parallel(aff, dec)[0], 1)
    # the product's own CPU frame decoder (mh_decode_frame_cpu: shader semantics to the
    # raster, block rows over threads) -- informational, not the baseline
    import metalhuffman_amd as mh
    for n, key in ((1, "product_cpu_frame_decoder_1thread_MBps"), (share, "product_cpu_frame_decoder_MBps")):
        mh.decode_frame_cpu(efs[0], n)
        reps = 4 if n == 1 else 32
        t0 = time.perf_counter()
        for i in range(reps):
            mh.decode_frame_cpu(efs[i % len(efs)], n)
        out[key] = round(reps * px / (time.perf_counter() - t0) / 1e6, 1)
    return out


def _free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# --------------------------------------------------------------------------------------
def main(argv=None) -> int:
    args = parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    use_dist = world > 1 or args.dist
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    # MH_BENCH_BACKEND=gloo rehearses the multi-rank path on a one-GPU box (every
    # rank on the same device, CPU collectives); the driver's runs use RCCL
    backend = os.environ.get("MH_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    # host waits spin (hipDeviceScheduleSpin) instead of yielding: the timed region's
    # closing synchronize wakes without a scheduler round trip (single-shot 20-step
    # walls: 138-147 us spin vs 141-177 us auto on one box, scripts/diag_timed_spread.sh).
    # Set on this rank's device before its context.
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    if hip.hipSetDevice(ctypes.c_int(local)) == 0:
        hip.hipSetDeviceFlags(ctypes.c_uint(1))
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a HIP device")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if use_dist:
        if world == 1:  # --dist on one GPU: a one-rank group on the loopback address
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    import metalhuffman_amd as mh
    import metalhuffman_amd.build as B
    if not os.path.exists(mh.LIB_PATH):
        B.build()
    from metalhuffman_amd import decoder as D
    from metalhuffman_amd import dist as MD
    from metalhuffman_amd import frames as F

    bb = F.bigbridge()
    # shared table: built on rank 0, broadcast over RCCL
    t_bcast_us = None
    if use_dist:
        # 256-byte canonical header over RCCL; each GPU builds T1/T2 + its decode table
        canon = mh.encode_frame(bb).canon if rank == 0 else None
        # the first broadcast also creates the communicator and loads the table-build
        # kernel; the second one is timed
        MD.broadcast_header_device_tables(canon, src=0, device=dev).check_status()
        torch.cuda.synchronize(dev)
        dist.barrier()
        tb = time.perf_counter()
        tables = MD.broadcast_header_device_tables(canon, src=0, device=dev)
        torch.cuda.synchronize(dev)
        t_bcast_us = (time.perf_counter() - tb) * 1e6
        tables.check_status()
    else:
        t1, t2 = mh.encode_frame(bb).tables()
        tables = D.DeviceTables.upload(t1, t2, dev)
    t2_bytes = 2 * tables.check_status()  # used T2 bytes (a device-built T2 keeps full capacity)

    # this rank's resident frames (distinct block shuffles: one shared table)
    seeds = [rank * args.frames + i for i in range(args.frames)]
    imgs = [F.block_shuffle(bb, s) for s in seeds]
    efs = encode_many(imgs)
    for ef in efs:
        assert np.array_equal(ef.canon, efs[0].canon)
    dimgs = torch.from_numpy(np.stack(imgs)).to(dev)  # the inputs, for the parity guard

    def pack(group):
        return D.DeviceFrames.pack(group, dev)

    def frame_workload():
        launches = [pack([ef]) for ef in efs]
        return Workload("frame", launches, tables, bb.size, algo_bytes(efs[:1], t2_bytes), dev,
                        refs=[dimgs[i:i + 1] for i in range(len(efs))],
                        read_bytes=algo_read_bytes(efs[:1], t2_bytes))

    def batch_workload(nb):
        starts = [i for i in range(0, len(efs), nb) if i + nb <= len(efs)] or [0]
        groups = [efs[i:i + nb] for i in starts]
        launches = [pack(g) for g in groups]
        return Workload(f"batch{nb}", launches, tables, nb * bb.size, algo_bytes(groups[0], t2_bytes), dev,
                        refs=[dimgs[i:i + nb] for i in starts],
                        read_bytes=algo_read_bytes(groups[0], t2_bytes))

    def tile_workload(random=False):
        # config 3: BigBridge mirror tile (primary) or uniform random bytes (stress:
        # 8 bits/symbol, every code 8 bits, no T2 subtable), SURVEY.md 8(d)
        base = F.uniform_random(8192, 8192, 1234) if random else F.mirror_tile(bb, 8192, 8192)
        # 6 distinct frames (680 MB of codes + offsets + rasters): a launch's inputs
        # were last touched 5 launches earlier, far past the 256 MiB Infinity Cache
        imgs = [base] + [F.block_shuffle(base, 100 + k) for k in range(TILE_FRAMES - 1)]
        tefs = encode_many(imgs, threads=TILE_FRAMES)
        t1t, t2t = tefs[0].tables()
        ttabs = D.DeviceTables.upload(t1t, t2t, dev)
        launches = [pack([ef]) for ef in tefs]
        name = "tile8192_random" if random else "tile8192"
        return Workload(name, launches, ttabs, base.size, algo_bytes(tefs[:1], ttabs.table2.numel()), dev,
                        refs=[torch.from_numpy(im).to(dev).unsqueeze(0) for im in imgs],
                        read_bytes=algo_read_bytes(tefs[:1], ttabs.table2.numel()))

    if args.workload == "frame":
        wl = frame_workload()
        wdesc = "config2: one 2048x1536 BigBridge-derived frame per launch per GPU"
    elif args.workload == "batch":
        wl = batch_workload(args.batch)
        wdesc = f"config4 shard: {args.batch} 2048x1536 frames per launch per GPU"
    elif args.workload == "tile8192":
        wl = tile_workload()
        wdesc = "config3: one 8192x8192 BigBridge mirror-tile per launch per GPU"
    else:
        wl = tile_workload(random=True)
        wdesc = "config3 stress: one 8192x8192 uniform-random frame per launch per GPU"

    # parity guard: every resident frame of every launch, before timing
    frames_verified = wl.verify()
    ref_shape = wl.refs[0].shape[1:]
    # multi-rank: every rank's verified-frame count gathered on rank 0
    ranks_ok = None
    rank_devices = None
    if use_dist:
        # self-proving multi-GPU run: each rank's HIP ordinal and
        # PCI bus id travel with its verified-frame count; under RCCL the (host, bus id)
        # pairs must be distinct, i.e. N ranks on N physical GPUs
        pci = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(pci, ctypes.c_int(64), ctypes.c_int(local)) != 0:
            raise SystemExit(f"rank {rank}: hipDeviceGetPCIBusId failed")
        me = {"rank": rank, "ordinal": int(torch.cuda.current_device()), "pci": pci.value.decode(),
              "host": socket.gethostname()}
        got = [None] * world
        dist.all_gather_object(got, (frames_verified, sum(f.n_frames for f in wl.launches), me))
        devs = {(g[2]["host"], g[2]["pci"]) for g in got}
        if backend == "nccl" and len(devs) != world:
            raise SystemExit(f"ranks share a GPU: {[g[2] for g in got]}")
        ranks_ok = sum(1 for a, b, _ in got if a == b) if len(devs) == world or backend != "nccl" else 0
        rank_devices = {"devices": [{k: g[2][k] for k in ("rank", "ordinal", "pci")} for g in got],
                        "distinct_devices": len(devs), "backend": backend}

    wall, region_ms, kms = wl.run(args.steps, args.warmup, use_graph=not args.no_graph, world=world)
    wl.check_outputs()  # the any-order / rotated regions' rasters
    per_step = wall / args.steps
    if not use_dist and not args.no_extras:
        ACHIEVABLE.update(hbm_probe() or {})  # after the timed region: the roofline context
    value = world * wl.pixels / per_step / 1e6

    result = {
        "metric": METRIC, "value": round(value, 1), "unit": "MB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(per_step * 1e3, 5),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: block-shuffled BigBridge.png (reference TEST_IMAGE4 asset), "
                f"{args.frames} distinct frames resident per GPU, shared canonical table",
        "config": {"workload": wdesc, "width": int(ref_shape[1]), "height": int(ref_shape[0]),
                   "frames_per_step_per_gpu": int(wl.launches[0].n_frames),
                   "parallelism": f"frame-sharded x{world}", "launch": wl.timed_launch},
        "mpixels_per_s": round(value, 1),
        "roofline": roofline(wl.bytes, region_ms, args.steps, kms, args.workload, wl.read_bytes,
                             wl.kernel_ms, wl.steady_kernel_ms, wl.steady_unit),
        "gpu_region_ms_per_step": round(region_ms / args.steps, 5),
        "timing": ("gated: the K launches are enqueued behind a host-opened launch gate before "
                   "the clock starts (scripts/micro/launch_gate.hip); every decode runs inside "
                   "the timed region" if wl.ungated_wall is not None else "plain"),
    }
    if wl.warm_wall is not None:
        # the clocked region re-decodes the launches the region before it just decoded,
        # no flush (still cache-resident for one-frame launches; not for the long
        # launches, whose launch sets cycle: see the docstring)
        result["warm_ms_per_step"] = round(wl.warm_wall / args.steps * 1e3, 5)
        result["warm_value"] = round(world * wl.pixels / (wl.warm_wall / args.steps) / 1e6, 1)
    if wl.ungated_wall is not None:
        # the same K launches timed the plain way (enqueue latency inside the clock)
        result["ungated_ms_per_step"] = round(wl.ungated_wall / args.steps * 1e3, 5)
        result["ungated_value"] = round(world * wl.pixels / (wl.ungated_wall / args.steps) / 1e6, 1)
    result["frames_verified"] = frames_verified
    # the sources this library was built from (the loader refuses a stale library)
    result["source_stamp"] = dict(B.source_stamps(), loaded=mh.lib().mh_build_stamp().decode()[:16])
    if ranks_ok is not None:
        result["ranks_verified"] = ranks_ok
        result["rank_devices"] = rank_devices
    if t_bcast_us is not None:
        result["table_broadcast_us"] = round(t_bcast_us, 1)  # 256-B RCCL broadcast + device table build
        result["table_broadcast_bytes"] = 256

    if not use_dist and rank == 0 and not args.no_extras:
        extras = {}
        if args.workload == "frame":
            # config 2 with independent frames in flight on several streams (one launch
            # per frame still): not `value`, which keeps one stream
            fs = {}
            for ns in (2, 4):
                per = wl.run_streams(args.steps, ns)
                if per:
                    fs[f"{ns}_streams"] = {"us_per_frame": round(per * 1e6, 3),
                                           "value_MBps": round(wl.pixels / per / 1e6, 1)}
            if fs:
                fs["method"] = (f"{args.steps} one-frame launches round-robined over the streams, "
                                "queued behind one launch gate per stream, best of 3 regions")
                extras["frame_streams"] = fs
        # ~20 ms of launches each, after a warm-up of the same length (clocks settle)
        for name, make, steps, key in (("batch64", lambda: batch_workload(args.batch), 256, "batch"),
                                       ("tile8192", tile_workload, 512, "tile8192"),
                                       ("tile8192_random", lambda: tile_workload(True), 512,
                                        "tile8192_random")):
            if name.startswith("batch") and args.workload == "batch":
                continue
            if name == args.workload:
                continue
            w2 = make()
            nver = w2.verify()
            wall2, reg2, kms2 = w2.run(steps, steps, use_graph=not args.no_graph)
            w2.check_outputs()
            extras[name] = {"value_MBps": round(w2.pixels / (wall2 / steps) / 1e6, 1),
                            "warm_value_MBps": (round(w2.pixels / (w2.warm_wall / steps) / 1e6, 1)
                                                if w2.warm_wall else None),
                            "ms_per_step": round(wall2 / steps * 1e3, 4),
                            "gpu_region_ms_per_step": round(reg2 / steps, 4),
                            "frames_verified": nver,
                            "roofline": roofline(w2.bytes, reg2, steps, kms2, key, w2.read_bytes,
                                                 w2.kernel_ms, w2.steady_kernel_ms, w2.steady_unit)}
            del w2
        extras["hbm_copy"] = copy_bandwidth(dev)  # achievable HBM rate beside the 8 TB/s spec
        if ACHIEVABLE:
            extras["hbm_probe"] = dict(ACHIEVABLE)
        extras["stream_h2d"] = stream_h2d(efs, tables, dev)  # config 5, one GPU
        extras["encode"] = encode_rate(dev, bb)
        result["extras"] = extras

    if use_dist and not args.no_extras:
        # The other multi-GPU configs on the same ranks (BASELINE configs[3], configs[4]):
        # config 4 = 64 frames per launch per GPU, timed like the headline (barrier +
        # synchronize, max over ranks); config 5 = every rank streaming host-resident
        # frames through its own mh_stream at once, so the node's shared host PCIe and
        # memory bandwidth is in the measurement.
        extras = {}
        b = batch_workload(args.batch)
        nver = b.verify()
        bsteps = 64
        bwall, breg, bkms = b.run(bsteps, 16, use_graph=not args.no_graph, world=world)
        extras["config4"] = {
            "frames_per_launch_per_gpu": int(b.launches[0].n_frames), "frames_total": world * int(b.launches[0].n_frames),
            "steps": bsteps, "value_MBps": round(world * b.pixels / (bwall / bsteps) / 1e6, 1),
            "ms_per_step": round(bwall / bsteps * 1e3, 4), "frames_verified_rank0": nver,
            "roofline_rank0": roofline(b.bytes, breg, bsteps, bkms, "batch", b.read_bytes, b.kernel_ms,
                                       b.steady_kernel_ms, b.steady_unit)}
        del b
        st = stream_h2d(efs, tables, dev, sync=dist.barrier)
        got = [None] * world
        dist.all_gather_object(got, {k: st[k] for k in ("fps", "h2d_GBps", "latency_us_p99", "latency_us_max",
                                                        "cold_fps")})
        extras["stream_h2d_all_ranks"] = {
            "ranks": world, "fps_sum": round(sum(g["fps"] for g in got), 1),
            "fps_min_rank": round(min(g["fps"] for g in got), 1),
            "value_MBps_incl_pcie": round(sum(g["fps"] for g in got) * bb.size / 1e6, 1),
            "h2d_GBps_sum": round(sum(g["h2d_GBps"] for g in got), 2),
            "cold_fps_min_rank": round(min(g["cold_fps"] for g in got), 1),
            "paced_latency_us_p99_max_rank": max(g["latency_us_p99"] for g in got),
            "paced_latency_us_max": max(g["latency_us_max"] for g in got),
            "method": "each rank: native mh_stream (2 slots), sustained phase started together after a barrier"}
        result["extras"] = extras

    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(efs[: min(len(efs), 32)], args.cpu_threads or None)

    if rank == 0:
        print(json.dumps(result), flush=True)
    if use_dist:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

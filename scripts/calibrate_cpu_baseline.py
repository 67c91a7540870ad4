"""Calibration of bench.py's cpu_baseline (kind "port") against the reference binary.

SURVEY.md section 6 timed the reference's own HuffmanUtil::decodeHuffmanBitsFromTables
(Shared/HuffmanUtil.cpp:830-1046, g++ -O2, BigBridge, one thread) at 105.7 MB/s in this
build container, during the survey. The reference's HuffmanUtil.cpp cannot be built here
any more without a stand-in for Apple's <simd/simd.h>, so the ratio is taken
against that recorded number: this script times the oracle restatement
(oracle/mh_oracle.c, the code cpu_baseline runs) exactly as cpu_baseline times its
one-thread leg, on the same frame, in the same container.

    python scripts/calibrate_cpu_baseline.py [reps]

Prints MB/s per trial and the median; ratio = port / reference (> 1: the port is faster
than the reference binary on the same core, so box numbers over-state the reference by
that factor).

This container's CPU speed drifts between sessions (the same oracle build timed 109.8 MB/s
in the round-5 review and 90-93 MB/s in round 6), so the raw ratio mixes code speed with
machine speed. The drift is gauged with the reference code that DOES build here: the
reference encoder (oracle/_ref/ref_encode, HuffmanEncoder.cpp compiled unmodified), which
SURVEY.md section 6 timed at 1.639 s on the 8192^2 tile in the survey session. drift =
t_now / 1.639 s; the drift-corrected ratio = port MB/s x drift / 105.7.
"""
from __future__ import annotations

import os
import platform
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

REFERENCE_MBPS = 105.7  # SURVEY.md section 6, reference binary, BigBridge, 1 thread, g++ -O2
REFERENCE_ENCODE_TILE_S = 1.639  # SURVEY.md section 6, reference encoder, 8192^2 tile, survey session


def main() -> int:
    from metalhuffman_amd import codec as C
    from metalhuffman_amd import frames as F
    from oracle import oracle as O

    O.build()
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    img = F.bigbridge()
    ef = C.encode_frame(img)
    t1, t2 = ef.tables()
    px = ef.width * ef.height
    nsym = ef.n_blocks * 64
    rates = []
    for _ in range(trials):
        sec = O.time_decode_frames(t1, t2, nsym, [ef.codes], 1, reps=16)
        rates.append(16 * px / sec / 1e6)
    med = statistics.median(rates)
    model = "?"
    with open("/proc/cpuinfo") as f:
        for line in f:
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    print(f"host {platform.node()} cpu {model}")
    print("port MB/s per trial:", [round(r, 1) for r in rates])
    print(f"port median {med:.1f} MB/s; reference (SURVEY 6) {REFERENCE_MBPS} MB/s; "
          f"raw ratio port/reference = {med / REFERENCE_MBPS:.3f}")
    if os.path.exists(O.REF_ENCODE):
        import subprocess
        import tempfile
        import time
        # the producer's symbols (Util.m:233-323 split, HuffmanUtil.cpp:21-85 per-block deltas)
        b = O.split_blocks(F.mirror_tile(img, 8192, 8192)).reshape(-1, 64).astype(np.int16)
        d = b.copy()
        d[:, 1:] = (b[:, 1:] - b[:, :-1]) & 0xFF
        sym = np.ascontiguousarray(d.astype(np.uint8)).reshape(-1)
        with tempfile.TemporaryDirectory() as d:
            src = os.path.join(d, "in.bin")
            sym.tofile(src)
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                subprocess.run([O.REF_ENCODE, src, "64", os.path.join(d, "out")], check=True,
                               stdout=subprocess.DEVNULL)
                ts.append(time.perf_counter() - t0)
        drift = min(ts) / REFERENCE_ENCODE_TILE_S
        print(f"reference encoder, 8192^2 tile: {[round(t, 3) for t in ts]} s (survey {REFERENCE_ENCODE_TILE_S} s): "
              f"machine drift {drift:.3f}")
        print(f"drift-corrected calibration_ratio port/reference = {med * drift / REFERENCE_MBPS:.3f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())

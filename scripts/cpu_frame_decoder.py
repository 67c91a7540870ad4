"""Host-core timing of the product's CPU frame decoder (mh_decode_frame_cpu) on one
2048x1536 BigBridge-shuffle frame: best of N calls at 1..16 threads, output checked.

Usage: python scripts/cpu_frame_decoder.py [reps]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import metalhuffman_amd as mh  # noqa: E402
from metalhuffman_amd import frames as F  # noqa: E402


def main() -> None:
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    img = F.block_shuffle(F.bigbridge(), 3)
    ef = mh.encode_frame(img)
    for n in (1, 2, 4, 8, 16):
        assert np.array_equal(mh.decode_frame_cpu(ef, n), img)
        best = 1e9
        for _ in range(reps):
            t0 = time.perf_counter()
            mh.decode_frame_cpu(ef, n)
            best = min(best, time.perf_counter() - t0)
        print(f"threads {n:2d}: {best * 1e3:7.3f} ms per frame, {img.size / best / 1e6:7.1f} MB/s", flush=True)


if __name__ == "__main__":
    main()

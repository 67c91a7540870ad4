"""CPU model (round 6): the single-frame kernel's first span fetched speculatively WITH the block
offsets, as a 5,120-byte window in the span registers (5 x 16 B per lane, what span_issue
already loads), placed from the linear guess guess(t) = frame bytes * t / tiles.

Round 5's model (scripts/model_spec_span.py) judged this negative: a tile whose true span is not
inside its window pays the exact second HBM round trip, and a launch ends with its slowest wave.
The difference modelled here: the four waves of a workgroup hold four consecutive tiles on one
XCD, so a miss's exact reload may already be in that XCD's L2 -- fetched by the neighbours'
windows issued at the same moment. Per workload this prints, per launch (frame):
  hit       the span is inside the wave's own window (no second round trip at all);
  l2        a miss whose span lies inside the union of its workgroup's four windows (the reload
            is an L2 round trip);
  hbm       any other miss (the reload is a second HBM round trip, as today);
and the extra HBM bytes the windows read beyond the spans they cover.

    python scripts/model_spec_window.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

WIN = 5120   # 5 chunks x 64 lanes x 16 B
WG = 4       # tiles per workgroup (small kernel)


def main() -> int:
    import metalhuffman_amd as mh
    from metalhuffman_amd import frames as F
    from model_spec_span import spans

    bb = F.bigbridge()
    work = {
        "bigbridge shuffles (bench config 2)": [F.block_shuffle(bb, s) for s in range(1, 9)],
        "bigbridge (natural)": [bb],
        "crop 777x1001": [F.crop(bb, 1001, 777)],
        "uniform random 2048x1536": [F.uniform_random(1536, 2048, 7)],
    }
    for lead in (1024, 1536, 2048):
        print(f"\nwindow {WIN} B starting {lead} B before the linear guess")
        for name, imgs in work.items():
            hit = l2 = hbm = 0
            waves = 0
            extra = []
            worst_hbm = 0
            for im in imgs:
                ef = mh.encode_frame(im)
                s, e, T = spans(ef)
                guess = (ef.payload_bytes * np.arange(T)) // T
                w0 = np.maximum(guess - lead, 0) & ~15
                w1 = w0 + WIN
                own = (s >= w0) & (e <= w1)
                # union of the workgroup's windows (contiguous: consecutive tiles' windows overlap)
                g = np.arange(T) // WG
                u0 = np.array([w0[g == k].min() for k in range(g.max() + 1)])[g]
                u1 = np.array([w1[g == k].max() for k in range(g.max() + 1)])[g]
                inwg = (~own) & (s >= u0) & (e <= u1)
                nh = int(np.sum(~own & ~inwg))
                hit += int(own.sum())
                l2 += int(inwg.sum())
                hbm += nh
                worst_hbm = max(worst_hbm, nh)
                waves += T
                # bytes read by windows that no span needs: window bytes outside [min s, max e) of the frame's spans
                covered = np.zeros(int(w1.max()) + 16, bool)
                for a, b in zip(s, e):
                    covered[a:b] = True
                fetched = np.zeros_like(covered)
                for a, b in zip(w0, w1):
                    fetched[a:b] = True
                extra.append(int(np.sum(fetched & ~covered)))
            print(f"  {name:38s} per launch: hit {hit / waves:6.1%}  l2 {l2 / waves:6.1%}  hbm {hbm / waves:6.2%} "
                  f"(worst launch {worst_hbm} of {T} waves); extra HBM bytes per launch {np.mean(extra) / 1e3:.0f} KB")
    return 0


if __name__ == "__main__":
    sys.exit(main())

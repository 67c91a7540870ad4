"""CPU model: a multi-symbol (pair) LUT for the BATCH kernel where lanes
that finish a block take the wave's next one, so the mean step count matters, not the max.

Reference semantics the table must keep: HuffmanUtil.cpp:338-667 (the split tables a pair
entry would be derived from) and huff_util.hpp:94-193 (canonical codes).

Per block, the pair step count comes from the real bitstream (scripts/model_pair_steps.py
`lookups`: a K-bit window decodes two codes when both fit). Three designs, per 64-block tile:
  today   one symbol per step, one lane per block: 64 wave-steps per tile (the step counts
          of the product's batch loop, PMC: 9.54 VALU, 4.25 SALU, 1.56 LDS per wave-step);
  fixed   pair steps, one lane per block: the tile runs until its slowest lane has 64 symbols;
  queue   pair steps, a wave owns a queue of Q tiles' blocks, a lane that finishes takes the
          next block after `switch` extra steps (its start offset, state reset, the block's
          rows flushed from LDS) -- wave-steps per tile = the queue's makespan / Q.
Per-step costs of a pair step (stated, not measured): +6 VALU (entry unpack, variable 1-2 byte
output position) and +1 LDS (the byte(s) into the lane's LDS row buffer; a lane's rows finish
at different steps, so they cannot be register-packed and stored per wave row as today).
LDS per 8-wave workgroup: pair table 2^K x 4 B (+ today's 2nd level) + per wave Q tile spans
(4,352 B each) + 64 x 64 B row buffer; today: 18,464 B + 8 x 4,352 B = 53 KB -> 3 per CU.

    python scripts/model_pair_queue.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

VALU, SALU, LDS = 9.54, 4.25, 1.56          # per wave-step today (profiles/r06_pmc_batch_head.txt)
PAIR_VALU, PAIR_LDS = 6.0, 1.0              # extra per pair step (model assumption)
SWITCH = 3                                   # extra steps when a lane takes a new block
LDS_CU = 160 * 1024


def queue_makespan(steps: np.ndarray, lanes: int = 64, switch: int = SWITCH) -> int:
    """Wave-steps to run `steps` (per block, in queue order) on `lanes` lanes, each lane
    taking the next block when its current one ends (plus `switch` steps)."""
    import heapq
    free = [0] * lanes  # time each lane becomes free
    heapq.heapify(free)
    end = 0
    first = True
    for i, s in enumerate(steps):
        t = heapq.heappop(free)
        cost = int(s) + (0 if i < lanes else switch)
        heapq.heappush(free, t + cost)
        end = max(end, t + cost)
        first = False
    return end


def occupancy(K: int, q: int) -> int:
    table = (1 << K) * 4 + 1040 * 2
    per_wave = q * 4352 + 64 * 64
    wg = table + 8 * per_wave
    return max(0, LDS_CU // wg)


def main() -> int:
    import metalhuffman_amd as mh
    from metalhuffman_amd import frames as F
    from model_pair_steps import lookups

    bb = F.bigbridge()
    cases = [("bigbridge shuffle (config 2/4 frame)", mh.encode_frame(F.block_shuffle(bb, 1))),
             ("8192^2 mirror tile, first 2048 rows (config 3)",
              mh.encode_frame(np.ascontiguousarray(F.mirror_tile(bb, 8192, 8192)[:2048])))]
    print(f"today: 64 wave-steps per tile = {64 * VALU:.0f} VALU, {64 * SALU:.0f} SALU, {64 * LDS:.0f} LDS per tile; "
          f"3 workgroups x 8 waves per CU")
    for K in (13, 14):
        for name, ef in cases:
            s = lookups(ef, K)
            nb = s.size - s.size % 64
            s = s[:nb]
            tiles = s.reshape(-1, 64)
            fixed = tiles.max(1).mean()
            print(f"\n{name}, K={K}: mean pair steps per block {s.mean():.1f} (today 64)")
            print(f"  fixed (max of 64 lanes): {fixed:5.1f} wave-steps per tile = {fixed / 64:.2f} of today's steps")
            for q in (1, 2, 4, 8):
                ms = [queue_makespan(s[i:i + 64 * q]) / q for i in range(0, nb - 64 * q + 1, 64 * q)]
                ws = float(np.mean(ms))
                valu = ws * (VALU + PAIR_VALU)
                lds = ws * (LDS + PAIR_LDS)
                occ = occupancy(K, q)
                print(f"  queue Q={q} tiles: {ws:5.1f} wave-steps per tile = {ws / 64:.2f} of today's steps; "
                      f"VALU {valu:6.0f} ({valu / (64 * VALU):.2f}x), LDS instr {lds:5.0f} ({lds / (64 * LDS):.2f}x); "
                      f"LDS budget -> {occ} workgroup(s) of 8 waves per CU (today 3)")
    print("\nReading: see profiles/r06_pair_queue_model.txt")
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""Round-6 forensics: run a batch-decode kernel from a hand-assembled code object.

Round 5's spilled batch-kernel build (commit 6793108's mh_decode.hip, 80 VGPRs + 40 B of
scratch) decoded symbol 5 of whole tiles wrongly in its flat-table loop. That loop's
ONLY 64-bit shift whose shift amount sits in v79 -- the last VGPR of an 80-VGPR
allocation -- is exactly step 5 of row 0. This script takes code objects assembled from
that build's device assembly, unchanged and with single-instruction patches
(scripts/forensic_isa_patch.sh makes them), loads each through hipModuleLoad and launches
its delta batch kernel on the uniform-random 8192^2 frame (the failing workload) with the
arguments mh_decode would pass, then counts wrong tiles.

    python scripts/forensic_isa_patch.py ab/isa_*.hsaco
"""
from __future__ import annotations

import ctypes
import os
import struct
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

KERNEL = b"_ZN12_GLOBAL__N_116mh_decode_kernelILb1EEEvNS_10DecodeArgsE"


def main() -> int:
    import torch
    from metalhuffman_amd import codec as C
    from metalhuffman_amd import decoder as D
    from metalhuffman_amd import frames as F

    hip = ctypes.CDLL("libamdhip64.so")
    dev = torch.device("cuda:0")
    img = F.uniform_random(8192, 8192, 1234)
    ef = C.encode_frame(img)
    t1, t2 = ef.tables()
    tabs = D.DeviceTables.upload(t1, t2, dev)
    fr = D.DeviceFrames.pack([ef], dev)
    torch.cuda.synchronize(dev)
    W = H = 8192
    bw = bh = 1024
    nb = bw * bh
    tiles = (nb + 63) // 64
    nwaves = 8
    n_groups = (tiles + nwaves - 1) // nwaves
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    grid = min(n_groups, cus * 3)  # 3 workgroups per CU (LDS), as hipOccupancy reports for this kernel
    out = torch.empty((H, W), dtype=torch.uint8, device=dev)
    ref = torch.from_numpy(img).to(dev)
    # DecodeArgs (6793108): 9 pointers / u64, 3 u64, then 12 u32 (t2_entries .. grid)
    args = struct.pack(
        "<QQQQQQQQQQQQ12I",
        fr.block_offsets.data_ptr(), fr.codes.data_ptr(), 0, fr.codes.numel(),
        tabs.table1.data_ptr(), tabs.table2.data_ptr(), tabs.lut.data_ptr(), 0,
        out.data_ptr(), W, 0, H * W,
        tabs.table2_entries, W, H, bw, bh, nb, tiles, tiles, n_groups, nwaves, grid, 0)
    args = args[: 12 * 8 + 11 * 4]
    args += b"\0" * ((-len(args)) % 8)
    print(f"grid {grid} x {nwaves * 64} threads, {tiles} tiles, gstride {grid * nwaves}, kernarg {len(args)} B",
          flush=True)
    for path in sys.argv[1:]:
        mod = ctypes.c_void_p()
        fn = ctypes.c_void_p()
        rc = hip.hipModuleLoad(ctypes.byref(mod), path.encode())
        rc = rc or hip.hipModuleGetFunction(ctypes.byref(fn), mod, KERNEL)
        if rc:
            print(path, "load failed", rc, flush=True)
            return 1
        buf = ctypes.create_string_buffer(args, len(args))
        size = ctypes.c_size_t(len(args))
        extra = (ctypes.c_void_p * 5)(ctypes.c_void_p(1), ctypes.cast(buf, ctypes.c_void_p),
                                      ctypes.c_void_p(2), ctypes.cast(ctypes.pointer(size), ctypes.c_void_p),
                                      ctypes.c_void_p(3))
        for rep in range(4):
            out.zero_()
            torch.cuda.synchronize(dev)
            rc = hip.hipModuleLaunchKernel(fn, grid, 1, 1, nwaves * 64, 1, 1, 0, None, None, extra)
            if rc:
                print(path, "launch failed", rc, flush=True)
                return 1
            torch.cuda.synchronize(dev)
            bad = (out != ref).view(bh, 8, bw, 8).permute(0, 2, 1, 3).reshape(nb, 64).any(dim=1)
            bad_tiles = torch.unique(torch.nonzero(bad).flatten() // 64).cpu().numpy()
            first = ""
            if bad_tiles.size:
                b = int(torch.nonzero(bad).flatten()[0])
                want = ref.view(bh, 8, bw, 8).permute(0, 2, 1, 3).reshape(nb, 64)[b].cpu().numpy()
                got = out.view(bh, 8, bw, 8).permute(0, 2, 1, 3).reshape(nb, 64)[b].cpu().numpy()
                first = f" first bad block {b}: first bad symbol {int(np.nonzero(want != got)[0][0])}"
            print(f"{os.path.basename(path)} rep {rep}: bad tiles {bad_tiles.size} of {tiles}{first}", flush=True)
        hip.hipModuleUnload(mod)
    return 0


if __name__ == "__main__":
    sys.exit(main())

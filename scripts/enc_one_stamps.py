"""Phase timestamps of the one-launch encoder (enc_one_kernel) on BigBridge frames.
Needs a library built with -DMH_CODE_STAMPS=1, loaded through MH_LIB:

    python -c "import metalhuffman_amd.build as B; B.build_variant('encstamps', ['MH_CODE_STAMPS=1'])"
    MH_LIB=ab/lib_encstamps.so python scripts/enc_one_stamps.py

Workgroup 0: [0] start, [3] hint counter complete, [4] tagged words summed, [1] every
tile's counts in, [2] table published.
Packing workgroup t+1: [0] start, [1] counts published, [2] table seen, [3] first bit
known (look-back), [4] tile written. Times in us from the earliest start (s_memrealtime,
100 MHz)."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from metalhuffman_amd import _native as N  # noqa: E402
from metalhuffman_amd import frames as F  # noqa: E402
from metalhuffman_amd.encoder import Encoder  # noqa: E402

L = N.lib()
L.mh_diag_code_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_size_t]
bb = F.bigbridge()
dev = torch.device("cuda:0")
img = torch.from_numpy(F.block_shuffle(bb, 901)).to(dev)
enc = Encoder(bb.shape[1], bb.shape[0], dev)
ntiles = (enc.nb + 127) // 128
for rep in range(4):
    L.mh_diag_code_stamps_reset()
    enc.encode_async(img)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (1024 * 8))()
    L.mh_diag_code_stamps(buf, 1024 * 8)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 8).astype(np.int64)[: ntiles + 1]
    t0 = a[:, 0][a[:, 0] > 0].min()
    us = lambda x: (x - t0) / 100.0
    w0 = a[0]
    pk = a[1:]
    pct = lambda v: "p0 %.1f p50 %.1f p100 %.1f" % (np.min(v), np.median(v), np.max(v))
    print(f"rep {rep}: wg0 start {us(w0[0]):.1f} hint-done {us(w0[3]):.1f} words-summed {us(w0[4]):.1f} "
          f"counts-in {us(w0[1]):.1f} table {us(w0[2]):.1f} | "
          f"packers start [{pct(us(pk[:, 0]))}] published [{pct(us(pk[:, 1]))}] table-seen "
          f"[{pct(us(pk[:, 2]))}] lookback [{pct(us(pk[:, 3]))}] written [{pct(us(pk[:, 4]))}]")

"""Phase timestamps of the two-launch encoder's code kernel (enc_code_kernel) and its
split kernel, BigBridge frame. Library built with -DMH_CODE_STAMPS=1 (MH_LIB):

    python -c "import metalhuffman_amd.build as B; B.build_variant('encstamps', ['MH_CODE_STAMPS=1'])"
    MH_LIB=ab/lib_encstamps.so python scripts/enc_two_stamps.py

Code kernel, workgroup 0 (tree): [0] start, [1] table stored, [3] end.
Packing workgroup t+1: [0] start, [1] flag seen (the earlier tiles' histograms already
summed before the wait), [2] table in LDS, [4] scan done, [5] packed, [6] written.
Times in us from the code kernel's earliest start (s_memrealtime, 100 MHz)."""
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
L.mh_diag_split_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_size_t]
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
    sb = (ctypes.c_ulonglong * (1024 * 8))()
    L.mh_diag_split_stamps(sb, 1024 * 8)
    sp = np.frombuffer(sb, dtype=np.uint64).reshape(1024, 8).astype(np.int64)[:ntiles]
    t0 = a[:, 0][a[:, 0] > 0].min()
    us = lambda x: (x - t0) / 100.0
    pk = a[1:]
    pct = lambda v: "p0 %.1f p50 %.1f p100 %.1f" % (np.min(v), np.median(v), np.max(v))
    print(f"rep {rep}: split [{pct(us(sp[:, 0]))}] -> [{pct(us(sp[:, 4]))}] | tree start {us(a[0, 0]):.1f} "
          f"table {us(a[0, 1]):.1f} end {us(a[0, 3]):.1f} | packers start [{pct(us(pk[:, 0]))}] flag-seen "
          f"[{pct(us(pk[:, 1]))}] tab [{pct(us(pk[:, 2]))}] scan [{pct(us(pk[:, 4]))}] "
          f"written [{pct(us(pk[:, 6]))}]")

"""Reentrancy (include/metalhuffman.h): two host threads decode at
the same time, each on its own HIP stream with its own tables, starting together on
a freshly loaded library so that both race through the per-device launch-parameter
initialisation (mh_decode.hip: std::call_once per device ordinal). The reference
keeps its decode tables in module statics (Shared/HuffmanUtil.cpp:87-102), which two
threads could not share; here every output must equal the oracle's decode."""
from __future__ import annotations

import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent(r"""
    import sys, threading
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    import metalhuffman_amd as mh
    from metalhuffman_amd import decoder as D
    from metalhuffman_amd import frames as F
    from oracle import oracle as O

    dev = torch.device("cuda", 0)
    bb = F.bigbridge()
    rnd = F.uniform_random(512, 640, 99)
    jobs = []
    for img in (bb, np.ascontiguousarray(bb[:777, :1001]), rnd,
                np.ascontiguousarray(F.mirror_tile(bb, 4096, 2048))):
        ef = mh.encode_frame(img)
        t1, t2 = ef.tables()
        want = O.decode_frame_shader(ef.block_offsets, ef.codes, t1, t2, ef.width, ef.height)
        assert np.array_equal(want, img)
        jobs.append((ef, t1, t2, img))
    # device buffers made before the threads start; the library's first mh_decode
    # call happens inside the threads, at the same time
    prepared = []
    for ef, t1, t2, img in jobs:
        prepared.append((D.DeviceTables.upload(t1, t2, dev), D.DeviceFrames.pack([ef], dev), img))
    torch.cuda.synchronize(dev)
    go = threading.Barrier(2)
    errors = []

    def worker(k):
        try:
            s = torch.cuda.Stream(dev)
            mine = prepared[k::2]
            outs = []
            go.wait()
            with torch.cuda.stream(s):
                for rep in range(25):
                    for tabs, fr, img in mine:
                        outs.append((D.decode(fr, tabs, stream=s), img, fr.width))
            s.synchronize()
            for out, img, w in outs:
                if not np.array_equal(out[0, :, :w].cpu().numpy(), img):
                    errors.append((k, img.shape))
        except Exception as e:
            errors.append((k, repr(e)))

    th = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    print("errors", errors)
    sys.exit(1 if errors else 0)
""").replace("ROOT", repr(ROOT))


@pytest.mark.timeout(240)
def test_two_threads_two_streams_fresh_library():
    r = subprocess.run([sys.executable, "-c", SCRIPT], cwd=ROOT, capture_output=True, text=True,
                       timeout=200)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    assert "errors []" in r.stdout

"""Multi-process decode on the GPU box's one GPU: 2 ranks (gloo rendezvous on
127.0.0.1, both on cuda:0) take rank 0's 256-byte canonical header, build T1/T2 and
the decode table ON the device (mh_build_tables_device) and decode their own frame
shard -- bench.py's multi-GPU path with gloo standing in for RCCL."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import metalhuffman_amd as mh
        from metalhuffman_amd import decoder as D
        from metalhuffman_amd import dist as MD
        from metalhuffman_amd import frames as F

        dev = torch.device("cuda", 0)
        bb = F.bigbridge()
        canon = mh.encode_frame(bb).canon if rank == 0 else None
        tabs = MD.broadcast_header_device_tables(canon, src=0, device=dev)
        tabs.check_status()
        lo, hi = MD.shard_range(6, world, rank)
        imgs = [F.block_shuffle(bb, 40 + f) for f in range(lo, hi)]
        efs = [mh.encode_frame(im) for im in imgs]
        out = D.decode(D.DeviceFrames.pack(efs, dev), tabs)
        torch.cuda.synchronize(dev)
        ok = all(np.array_equal(out[i, :, :2048].cpu().numpy(), im) for i, im in enumerate(imgs))
        q.put((rank, lo, hi, ok))
    except Exception as e:  # report instead of hanging the parent's queue.get
        q.put((rank, -1, -1, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_ranks_header_broadcast_device_tables():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == [(0, 0, 3, True), (1, 3, 6, True)]

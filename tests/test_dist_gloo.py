"""Multi-process path on CPU (gloo, world_size 2): frame sharding and the shared
symbol-table broadcast, the same code bench.py runs over RCCL on MI355X nodes."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


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
    sys.path.insert(0, os.path.join(root, "tests"))
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import metalhuffman_amd as mh
        from metalhuffman_amd import dist as MD
        from metalhuffman_amd import frames as F
        from oracle import oracle as O

        bb = np.ascontiguousarray(F.bigbridge()[:768, :1024])
        t1 = t2 = canon = None
        if rank == 0:
            ef0 = mh.encode_frame(bb)
            canon = ef0.canon
            t1, t2 = ef0.tables()
        d1, d2 = MD.broadcast_tables(t1, t2, src=0, device="cpu")
        c_all, r1, r2 = MD.broadcast_canonical_header(canon, src=0, device="cpu")
        n_frames = 7
        lo, hi = MD.shard_range(n_frames, world, rank)
        ok = True
        for f in range(lo, hi):
            img = F.block_shuffle(bb, f)
            ef = mh.encode_frame(img)
            ok &= bool(np.array_equal(ef.canon, c_all))          # shared table holds
            out = O.decode_frame_shader(ef.block_offsets, ef.codes, d1.numpy(), d2.numpy(),
                                        ef.width, ef.height)
            ok &= bool(np.array_equal(out, img))
        q.put((rank, lo, hi, ok, d1.numpy().tobytes() + d2.numpy().tobytes(),
               r1.tobytes() + r2.tobytes()))
    except Exception as e:  # report instead of hanging the peer's queue.get
        q.put((rank, -1, -1, False, repr(e).encode(), b""))
        raise
    finally:
        dist.destroy_process_group()


def test_shard_range_partitions():
    from metalhuffman_amd.dist import shard_range
    for n in (0, 1, 7, 64, 512):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.timeout(300)
def test_gloo_world2_table_broadcast_and_shards():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, lo0, hi0, ok0, tab0, reb0), (r1, lo1, hi1, ok1, tab1, reb1) = res
    assert (lo0, hi0, lo1, hi1) == (0, 4, 4, 7)
    assert ok0 and ok1
    assert tab0 == tab1 == reb0 == reb1      # every rank holds rank 0's T1||T2


def _band_worker(rank, world, port, q):
    """Single-frame split: rank 0 encodes one frame and sends each rank only its
    band (offsets + code bytes); every rank decodes its rows, rank 0 gathers them."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import metalhuffman_amd as mh
        from metalhuffman_amd import dist as MD
        from metalhuffman_amd import frames as F
        from oracle import oracle as O

        img = np.ascontiguousarray(F.bigbridge()[:777, :1001])
        bands = [None] * world
        if rank == 0:
            ef = mh.encode_frame(img)
            bands = [MD.frame_band(ef, world, r) for r in range(world)]
        mine = [None]
        dist.scatter_object_list(mine, bands if rank == 0 else None, src=0)
        band, y0 = mine[0]
        t1, t2 = band.tables()
        rows = O.decode_frame_shader(band.block_offsets, band.codes, t1, t2, band.width, band.height)
        got = [None] * world
        dist.all_gather_object(got, (y0, rows, int(band.codes.size)))
        full = np.concatenate([g[1] for g in sorted(got, key=lambda g: g[0])])
        q.put((rank, bool(np.array_equal(full, img)), [g[2] for g in got]))
    except Exception as e:  # report instead of hanging the peer's queue.get
        q.put((rank, False, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_single_frame_split():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_band_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, ok0, sizes0), (_, ok1, sizes1) = res
    assert ok0 and ok1, (sizes0, sizes1)
    assert sizes0 == sizes1 and all(s > 0 for s in sizes0)

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


def _nccl_worker(port, q):
    """World size 1 over the real backend ("nccl" = RCCL on ROCm): the device-tensor
    branch of broadcast_header_device_tables, all_gather_object and an all_reduce
    on a device tensor -- the calls bench.py's multi-GPU path makes."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        import metalhuffman_amd as mh
        from metalhuffman_amd import decoder as D
        from metalhuffman_amd import dist as MD
        from metalhuffman_amd import frames as F

        assert dist.get_backend() == "nccl"
        bb = F.bigbridge()
        canon = mh.encode_frame(bb).canon
        tabs = MD.broadcast_header_device_tables(canon, src=0, device=dev)
        tabs.check_status()
        # T1 || T2 broadcast too (the alternative to the 256-byte header)
        t1, t2 = mh.encode_frame(bb).tables()
        bt1, bt2 = MD.broadcast_tables(t1, t2, src=0, device=dev)
        assert bt1.is_cuda and np.array_equal(bt1.cpu().numpy(), t1.view(np.uint8).ravel())
        imgs = [F.block_shuffle(bb, 70 + f) for f in range(3)]
        efs = [mh.encode_frame(im) for im in imgs]
        out = D.decode(D.DeviceFrames.pack(efs, dev), tabs)
        torch.cuda.synchronize(dev)
        ok = all(np.array_equal(out[i, :, :2048].cpu().numpy(), im) for i, im in enumerate(imgs))
        got = [None]
        dist.all_gather_object(got, (3, int(ok)))
        t = torch.tensor([1.5], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.barrier()
        q.put(("ok", ok, got[0], float(t.item())))
    except Exception as e:  # report instead of hanging the parent's queue.get
        q.put(("err", repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_rccl_world1_device_broadcast():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), q))
    p.start()
    try:
        res = q.get(timeout=240)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert res[0] == "ok", res
    assert res[1] is True and res[2] == (3, 1) and res[3] == 1.5
    assert p.exitcode == 0


@pytest.mark.timeout(300)
def test_bench_dist_path_on_rccl_world1():
    """bench.py --dist on the one-GPU box: the multi-GPU code path under RCCL at world
    size 1 -- 256-byte header broadcast into device memory, device table build, the
    max-over-ranks timing all_reduce, config 4 (a batch launch per rank) and config 5
    (every rank streaming) -- with the parity guard on every resident frame."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MH_BENCH_BACKEND="nccl")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--dist", "--steps", "8", "--warmup", "2",
                        "--frames", "8", "--batch", "8", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=280, cwd=root)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["frames_verified"] == 8 and line["ranks_verified"] == 1
    rd = line["rank_devices"]  # the line names each rank's GPU
    assert rd["backend"] == "nccl" and rd["distinct_devices"] == 1, rd
    assert rd["devices"][0]["rank"] == 0 and rd["devices"][0]["ordinal"] == 0, rd
    assert rd["devices"][0]["pci"].count(":") >= 2, rd
    assert line["table_broadcast_bytes"] == 256
    ex = line["extras"]
    assert ex["config4"]["frames_verified_rank0"] == 8
    assert ex["stream_h2d_all_ranks"]["ranks"] == 1 and ex["stream_h2d_all_ranks"]["fps_sum"] > 0

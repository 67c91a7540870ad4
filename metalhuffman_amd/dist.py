"""Multi-GPU layout: one process per GPU, frames sharded, the table broadcast once.

Frames are independent (each carries its own block offsets), so the batch is split
into contiguous per-rank frame ranges with no data-path collective. The only
exchange is the shared symbol table: rank 0 broadcasts the 256-byte canonical
header and every GPU rebuilds T1/T2 and its decode table on the device
(broadcast_header_device_tables), or rank 0 broadcasts T1||T2 itself (BigBridge:
512 + 14,848 bytes). With backend "nccl" on ROCm that is RCCL over xGMI; with
"gloo" (tests) it runs on the CPU.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from .codec import Huffman


def shard_range(n_items: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [lo, hi) share of n_items for `rank` (sizes differ by at most 1)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    base, extra = divmod(n_items, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def frame_band(ef, world: int, rank: int):
    """Single-frame split: `rank`'s contiguous share of the frame's
    block rows as a self-contained EncodedFrame (EncodedFrame.band) plus its first
    pixel row. Only that band's code bytes and offsets go to the rank; the decoded
    bands, stacked in rank order, are the frame."""
    by0, by1 = shard_range(ef.block_height, world, rank)
    if by0 == by1:
        return None, 8 * by0
    return ef.band(by0, by1), 8 * by0


def _bcast_bytes(payload: np.ndarray | None, src: int, device: torch.device, group=None) -> np.ndarray:
    rank = dist.get_rank(group)
    n = torch.zeros(1, dtype=torch.int64, device=device)
    if rank == src:
        n[0] = int(payload.size)
    dist.broadcast(n, src=src, group=group)
    buf = torch.empty(int(n.item()), dtype=torch.uint8, device=device)
    if rank == src:
        buf.copy_(torch.from_numpy(np.ascontiguousarray(payload, np.uint8)))
    dist.broadcast(buf, src=src, group=group)
    return buf


def broadcast_tables(t1: np.ndarray | None, t2: np.ndarray | None, src: int = 0,
                     device: torch.device | str = "cpu", group=None):
    """Broadcast T1||T2 from `src`; returns device tensors (t1, t2) on every rank."""
    device = torch.device(device)
    payload = None
    if dist.get_rank(group) == src:
        payload = np.concatenate([np.ascontiguousarray(t1, np.uint8), np.ascontiguousarray(t2, np.uint8)])
    buf = _bcast_bytes(payload, src, device, group)
    return buf[:512], buf[512:]


def broadcast_canonical_header(canon: np.ndarray | None, src: int = 0,
                               device: torch.device | str = "cpu", group=None):
    """Broadcast the 256-byte canonical header; every rank rebuilds T1/T2 itself
    (HuffmanUtil.cpp:270-310 + :338-667 via the host codec)."""
    device = torch.device(device)
    buf = _bcast_bytes(canon if dist.get_rank(group) == src else None, src, device, group)
    canon_all = buf.cpu().numpy()
    t1, t2 = Huffman.generateSplitLookupTables(canon_all)
    return canon_all, t1, t2


def broadcast_header_device_tables(canon: np.ndarray | None, src: int = 0,
                                   device: torch.device | str = "cuda", group=None):
    """Broadcast the 256-byte canonical header from `src` straight into device
    memory and build T1/T2 + the prepared decode table there
    (mh_build_tables_device): one 256-byte RCCL broadcast per table change."""
    from .decoder import DeviceTables
    device = torch.device(device)
    # RCCL broadcasts device memory; gloo (CPU tests) a host tensor
    on = device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    buf = torch.empty(256, dtype=torch.uint8, device=on)
    if dist.get_rank(group) == src:
        buf.copy_(torch.from_numpy(np.ascontiguousarray(canon, np.uint8)))
    dist.broadcast(buf, src=src, group=group)
    return DeviceTables.from_canonical_header(buf, device)

"""GPU decode path: torch device tensors in, W x H uint8 raster out, via mh_decode().

This is the host-side mirror of the reference renderer's decode contract
(Shared/AAPLRenderer.m:1192-1678): the same five buffers (block offsets, huffBuff,
T1, T2, dims) are uploaded once (the renderer's MTLBuffers, :576-667) and every
decode is one launch of the HIP kernel in csrc/mh_decode.hip. PyTorch is only the
device-memory / stream plumbing; nothing here computes on the CPU.
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import Optional, Sequence

import numpy as np
import torch

from . import _native as N
from .codec import EncodedFrame, block_grid

ALIGN = 16  # frame code starts inside a packed batch (16-byte buffer loads)


def _dev(device) -> torch.device:
    d = torch.device(device)
    if d.type != "cuda":
        raise RuntimeError("the MI355X decoder needs a HIP device (torch 'cuda' on ROCm)")
    if d.index is None:  # 'cuda' -> the current device, so device checks compare equal
        d = torch.device("cuda", torch.cuda.current_device())
    return d


def _stream_ptr(stream: Optional[torch.cuda.Stream], device: torch.device) -> int:
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return int(s.cuda_stream)


@dataclasses.dataclass
class DeviceTables:
    """T1/T2 (+ the derived LDS table) resident on one device."""
    table1: torch.Tensor     # u8[512]
    table2: torch.Tensor     # u8[2 * entries]
    lut: Optional[torch.Tensor]  # u8[mh_lut_bytes()] from mh_prepare_lut, or None

    @property
    def table2_entries(self) -> int:
        return self.table2.numel() // 2

    @classmethod
    def upload(cls, t1: np.ndarray, t2: np.ndarray, device="cuda", prepare_lut: bool = True,
               stream: Optional[torch.cuda.Stream] = None) -> "DeviceTables":
        dev = _dev(device)
        d1 = torch.from_numpy(np.ascontiguousarray(t1, np.uint8)).to(dev)
        d2 = torch.from_numpy(np.ascontiguousarray(t2, np.uint8)).to(dev)
        tabs = cls(d1, d2, None)
        if prepare_lut:
            tabs.prepare_lut(stream)
        return tabs

    @classmethod
    def from_canonical_header(cls, canon, device="cuda", prepare_lut: bool = True,
                              stream: Optional[torch.cuda.Stream] = None) -> "DeviceTables":
        """Build T1/T2 (and the prepared table) ON the device from the 256-byte
        canonical header (mh_build_tables_device), e.g. after a 256-byte broadcast.
        T2 keeps its full MH_TABLE2_MAX_ENTRIES capacity (zero past the used
        subtables). Asynchronous; check_status() syncs and raises on a bad header."""
        dev = _dev(device)
        if isinstance(canon, torch.Tensor):
            hdr = canon.to(dev, torch.uint8).contiguous()
        else:
            hdr = torch.from_numpy(np.ascontiguousarray(canon, np.uint8)).to(dev)
        if hdr.numel() != 256:
            raise ValueError("the canonical header has 256 entries")
        d1 = torch.empty(512, dtype=torch.uint8, device=dev)
        d2 = torch.empty(2 * N.MH_TABLE2_MAX_ENTRIES, dtype=torch.uint8, device=dev)
        meta = torch.zeros(2, dtype=torch.int32, device=dev)  # [used T2 entries, status]
        lut = torch.empty(int(N.lib().mh_lut_bytes()), dtype=torch.uint8, device=dev) if prepare_lut else None
        N.check(N.lib().mh_build_tables_device(hdr.data_ptr(), d1.data_ptr(), d2.data_ptr(),
                                               meta.data_ptr(), lut.data_ptr() if lut is not None else None,
                                               meta.data_ptr() + 4, _stream_ptr(stream, dev)),
                "mh_build_tables_device")
        tabs = cls(d1, d2, lut)
        tabs._meta = meta
        return tabs

    def check_status(self) -> int:
        """Used T2 entries of a device-built table (synchronises); raises MHError
        when the header was rejected."""
        meta = getattr(self, "_meta", None)
        if meta is None:
            return self.table2_entries
        entries, status = (int(v) for v in meta.cpu().tolist())
        N.check(status, "mh_build_tables_device")
        return entries

    def prepare_lut(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        dev = self.table1.device
        lut = torch.empty(int(N.lib().mh_lut_bytes()), dtype=torch.uint8, device=dev)
        N.check(N.lib().mh_prepare_lut(self.table1.data_ptr(), self.table2.data_ptr(),
                                       self.table2_entries, lut.data_ptr(),
                                       _stream_ptr(stream, dev)), "mh_prepare_lut")
        self.lut = lut


@dataclasses.dataclass
class DeviceFrames:
    """n frames of one size that share one table pair, packed for mh_decode."""
    width: int
    height: int
    n_frames: int
    block_offsets: torch.Tensor          # u32 as int32[n * NB]
    codes: torch.Tensor                  # u8[total]
    frame_code_offsets: Optional[torch.Tensor]  # int64[n + 1] (None for one frame)
    block_init: Optional[torch.Tensor] = None   # u8[n * NB]
    flags: int = 0
    code_bytes: int = 0                  # payload bytes (sum over frames, pad excluded)

    @property
    def n_blocks(self) -> int:
        bw, bh = block_grid(self.width, self.height)
        return bw * bh

    @classmethod
    def pack(cls, frames: Sequence[EncodedFrame], device="cuda") -> "DeviceFrames":
        """Upload frames (host arrays) into one packed device batch."""
        dev = _dev(device)
        if not frames:
            raise ValueError("no frames")
        w, h, fl = frames[0].width, frames[0].height, frames[0].flags
        for f in frames:
            if (f.width, f.height, f.flags) != (w, h, fl):
                raise ValueError("a batch holds frames of one size and one format")
            if not np.array_equal(f.canon, frames[0].canon):
                raise ValueError("a batch shares one canonical table")
        starts = [0]
        for f in frames:
            starts.append(starts[-1] + ((f.codes.size + ALIGN - 1) // ALIGN) * ALIGN)
        packed = np.zeros(starts[-1], np.uint8)
        for f, s in zip(frames, starts):
            packed[s: s + f.codes.size] = f.codes
        offs = np.concatenate([f.block_offsets for f in frames]).astype(np.uint32)
        init = None
        if frames[0].block_init is not None:
            init = torch.from_numpy(np.concatenate([f.block_init for f in frames])).to(dev)
        fco = None
        if len(frames) > 1:
            fco = torch.tensor(starts, dtype=torch.int64, device=dev)
        return cls(w, h, len(frames), torch.from_numpy(offs.view(np.int32)).to(dev),
                   torch.from_numpy(packed).to(dev), fco, init, fl,
                   sum(f.payload_bytes for f in frames))


def _frame_entry(frames: DeviceFrames, tables: DeviceTables, extra_flags: int = 0):
    """(mh_frame, device index) for (frames, tables), extra_flags ORed into the frames'
    flags. Filling a ctypes struct field by field costs ~5.5 us of Python -- more than
    the 5.3 us decode of a 2048x1536 frame -- so the structs are kept on `frames` and
    reused while the buffers and sizes they were built from are the same objects (the
    buffer tensors are the renderer's MTLBuffers: allocated once, never re-seated in
    place; the cache holds references to them, so their ids cannot be reused). The
    device check runs when an entry is built. Callers never modify the struct."""
    refs = (frames.block_offsets, frames.codes, frames.frame_code_offsets, frames.block_init,
            tables.table1, tables.table2, tables.lut)
    key = (id(refs[0]), id(refs[1]), id(refs[2]), id(refs[3]), id(refs[4]), id(refs[5]), id(refs[6]),
           frames.width, frames.height, frames.n_frames, frames.flags)
    cache = frames.__dict__.get("_fr_cache")
    if cache is None or cache[0] != key:
        dev = frames.codes.device
        if dev.type != "cuda" or any(t is not None and t.device != dev for t in refs):
            raise ValueError("tables and frames must live on the same HIP device")
        cache = (key, refs, {}, dev.index)
        frames.__dict__["_fr_cache"] = cache
    fr = cache[2].get(extra_flags)
    if fr is None:
        bw, bh = block_grid(frames.width, frames.height)
        ptr = [t.data_ptr() if t is not None else None for t in refs]
        fr = N.mh_frame(ptr[0], ptr[1], frames.codes.numel(), ptr[2], ptr[4], ptr[5],
                        tables.table2_entries, ptr[6], ptr[3],
                        N.mh_dims(frames.width, frames.height, bw, bh), frames.n_frames,
                        frames.flags | extra_flags)
        cache[2][extra_flags] = fr
    return fr, cache[3]


def _frame_struct(frames: DeviceFrames, tables: DeviceTables, extra_flags: int = 0) -> N.mh_frame:
    return _frame_entry(frames, tables, extra_flags)[0]


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def decode(frames: DeviceFrames, tables: DeviceTables, out: Optional[torch.Tensor] = None,
           stream: Optional[torch.cuda.Stream] = None, extra_flags: int = 0) -> torch.Tensor:
    """Decode every frame into out[n, H, pitch] (pitch = W rounded up to 8).
    extra_flags: decode-only flags ORed into the frame's (MH_FLAG_ANY_ORDER; MH_FLAG_LANE_PAIRS
    routes the call to the lane-pair diagnostic library, _native.diag_lanepairs()).
    The per-call host path is kept lean (a cached struct, the raw current stream): one
    frame decodes in ~5.3 us, so every microsecond of Python shows in eager loops."""
    fr, dev_index = _frame_entry(frames, tables, extra_flags)
    pitch = (frames.width + 7) // 8 * 8
    h = frames.height
    if out is None:
        out = torch.empty((frames.n_frames, h, pitch), dtype=torch.uint8, device=frames.codes.device)
    else:
        sh = out.shape
        if (out.dtype is not torch.uint8 or len(sh) < 2 or sh[-1] != pitch or sh[-2] != h
                or out.get_device() != dev_index or not out.is_contiguous()
                or out.numel() < frames.n_frames * h * pitch):
            raise ValueError(f"out must be a contiguous uint8 [{frames.n_frames}, {h}, {pitch}] "
                             f"tensor on cuda:{dev_index}")
    if stream is not None:
        sp = stream.cuda_stream
    elif _raw_stream is not None:
        sp = _raw_stream(dev_index)
    else:
        sp = torch.cuda.current_stream(dev_index).cuda_stream
    if fr.flags & N.MH_FLAG_LANE_PAIRS:  # the diagnostic library's kernel (A/B only)
        rc = N.diag_lanepairs().mh_diag_decode_lanepairs(ctypes.byref(fr), out.data_ptr(), pitch, h * pitch, sp)
    else:
        rc = N.lib().mh_decode(ctypes.byref(fr), out.data_ptr(), pitch, h * pitch, sp)
    if rc:
        N.check(rc, "mh_decode")
    return out


CHECK_FIELDS = ("zero_width_lookups", "bad_escapes", "length_mismatches", "first_bad_block")


def check(frames: DeviceFrames, tables: DeviceTables,
          stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
    """Debug mode of the decode contract (mh_check): per frame u32[4] =
    (zero-width lookups, T1 escapes past T2, blocks whose codes miss the next
    block's offset, first offending block or 0xFFFFFFFF), as an int64 tensor
    [n_frames, 4] on the device. Never touches a raster."""
    dev = frames.codes.device
    rep = torch.empty((frames.n_frames, 4), dtype=torch.int32, device=dev)
    fr = _frame_struct(frames, tables)
    N.check(N.lib().mh_check(ctypes.byref(fr), rep.data_ptr(), _stream_ptr(stream, dev)), "mh_check")
    return rep.to(torch.int64) & 0xFFFFFFFF


def decode_frames(encoded: Sequence[EncodedFrame], device="cuda") -> np.ndarray:
    """Convenience: upload, decode, copy back; returns [n, H, W] uint8 on the host."""
    t1, t2 = encoded[0].tables()
    tabs = DeviceTables.upload(t1, t2, device)
    frames = DeviceFrames.pack(encoded, device)
    out = decode(frames, tabs)
    return out[..., : frames.width].cpu().numpy()

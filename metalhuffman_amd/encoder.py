"""GPU encoder: a device frame in, the reference's buffers out (mh_encode_frame_device).

Byte-identical to the host codec (codec.encode_frame), so frames encoded on the GPU
feed the decoder -- and the reference's own renderer contract -- unchanged.
Encoder.encode returns the header and byte count on the host (one synchronisation);
Encoder.encode_async (mh_encode_frame_device_async) leaves everything on the device,
so an encode -> table build -> decode chain never waits on the host.
"""
from __future__ import annotations

import contextlib
import ctypes
import dataclasses
from typing import Optional

import numpy as np
import torch

from . import _native as N
from .codec import block_grid
from .decoder import DeviceFrames, _dev, _stream_ptr


@dataclasses.dataclass
class DeviceEncodedFrame:
    width: int
    height: int
    canon: np.ndarray                 # u8[256] canonical header (host)
    codes: torch.Tensor               # u8[codes_len] on the device (payload + 4 zero bytes)
    block_offsets: torch.Tensor       # int32 view of u32[NB] on the device
    block_init: Optional[torch.Tensor]
    flags: int

    @property
    def payload_bytes(self) -> int:
        return int(self.codes.numel()) - N.MH_CODES_PAD

    def frames(self) -> DeviceFrames:
        """The encoded frame as a one-frame DeviceFrames for decode()."""
        return DeviceFrames(self.width, self.height, 1, self.block_offsets, self.codes, None,
                            self.block_init, self.flags, self.payload_bytes)


class Encoder:
    """Reusable device workspace + output buffers for frames of one size. Calls on
    one stream queue up behind each other; frames in flight on several streams need
    one Encoder (one workspace) per stream."""

    def __init__(self, width: int, height: int, device="cuda"):
        self.device = _dev(device)
        self.width, self.height = width, height
        bw, bh = block_grid(width, height)
        self.nb = bw * bh
        ws = int(N.lib().mh_encode_workspace_bytes(width, height))
        # zero-filled once: every encode leaves the histogram zeroed for the next, so
        # the calls pass MH_ENCODE_WORKSPACE_ZEROED and skip the per-call clear
        self.workspace = torch.zeros(ws + 256, dtype=torch.uint8, device=self.device)
        self.cap = (self.nb * 64 * 2 + N.MH_CODES_PAD + 3) // 4 * 4 + 16

    def encode(self, gray: torch.Tensor, flags: int = 0, init_zero_delta: bool = False,
               stream: Optional[torch.cuda.Stream] = None) -> DeviceEncodedFrame:
        if gray.dtype != torch.uint8 or gray.shape != (self.height, self.width) or not gray.is_contiguous():
            raise ValueError(f"gray must be contiguous uint8 [{self.height}, {self.width}]")
        gray = gray.to(self.device)
        codes = torch.empty(self.cap, dtype=torch.uint8, device=self.device)
        offs = torch.empty(self.nb, dtype=torch.int32, device=self.device)
        init = torch.empty(self.nb, dtype=torch.uint8, device=self.device) if init_zero_delta else None
        canon = np.zeros(256, np.uint8)
        n = ctypes.c_uint64(0)
        base = self.workspace.data_ptr()
        aligned = (base + 255) // 256 * 256
        N.check(N.lib().mh_encode_frame_device(
            gray.data_ptr(), self.width, self.height, flags | N.MH_ENCODE_WORKSPACE_ZEROED,
            canon.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), codes.data_ptr(), self.cap,
            ctypes.byref(n), offs.data_ptr(), init.data_ptr() if init is not None else None,
            aligned, self.workspace.numel() - (aligned - base), _stream_ptr(stream, self.device)),
            "mh_encode_frame_device")
        return DeviceEncodedFrame(self.width, self.height, canon, codes[: n.value], offs, init, flags)

    def encode_async(self, gray: torch.Tensor, flags: int = 0, init_zero_delta: bool = False,
                     stream: Optional[torch.cuda.Stream] = None,
                     codes: Optional[torch.Tensor] = None) -> AsyncEncodedFrame:
        """Enqueue the encode on `stream` (default: the current stream) and return
        at once. `gray` must be ready on that stream (make it wait on the stream
        that produced the frame). `codes` may be a reused u8 buffer of at least the
        encoder's capacity (the default allocates one)."""
        if gray.dtype != torch.uint8 or gray.shape != (self.height, self.width) or not gray.is_contiguous():
            raise ValueError(f"gray must be contiguous uint8 [{self.height}, {self.width}]")
        if gray.device != self.device:
            raise ValueError("gray must live on the encoder's device")
        # outputs belong to the stream the kernels run on (the caching allocator must
        # not hand their memory out again while that stream still writes it)
        with torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext():
            if codes is None:
                codes = torch.empty(self.cap, dtype=torch.uint8, device=self.device)
            offs = torch.empty(self.nb, dtype=torch.int32, device=self.device)
            init = torch.empty(self.nb, dtype=torch.uint8, device=self.device) if init_zero_delta else None
            canon = torch.empty(256, dtype=torch.uint8, device=self.device)
            meta = torch.empty(2, dtype=torch.int64, device=self.device)   # [codes_len, status]
        if codes.dtype != torch.uint8 or codes.device != self.device or codes.numel() < 4:
            raise ValueError("codes must be a uint8 buffer on the encoder's device")
        base = self.workspace.data_ptr()
        aligned = (base + 255) // 256 * 256
        N.check(N.lib().mh_encode_frame_device_async(
            gray.data_ptr(), self.width, self.height, flags | N.MH_ENCODE_WORKSPACE_ZEROED,
            canon.data_ptr(), codes.data_ptr(),
            codes.numel(), meta.data_ptr(), offs.data_ptr(), init.data_ptr() if init is not None else None,
            meta.data_ptr() + 8, aligned, self.workspace.numel() - (aligned - base),
            _stream_ptr(stream, self.device)), "mh_encode_frame_device_async")
        return AsyncEncodedFrame(self.width, self.height, canon, codes, meta[0:1],
                                 meta[1:2].view(torch.int32)[0:1], offs, init, flags)


@dataclasses.dataclass
class AsyncEncodedFrame:
    """An encode still in flight on the device: header, byte count and status are
    device tensors. frames()/tables() chain the decode without a host sync;
    result() synchronises and returns the DeviceEncodedFrame (raising MHError on
    a rejected frame)."""
    width: int
    height: int
    canon: torch.Tensor               # u8[256] on the device
    codes: torch.Tensor               # u8[capacity] on the device (first codes_len bytes used)
    codes_len: torch.Tensor           # int64[1] on the device (0 on an error)
    status: torch.Tensor              # int32[1] on the device
    block_offsets: torch.Tensor
    block_init: Optional[torch.Tensor]
    flags: int

    def frames(self) -> DeviceFrames:
        """A one-frame DeviceFrames over the whole code buffer (the decoder bounds
        the last block by its offset, not by the buffer size)."""
        return DeviceFrames(self.width, self.height, 1, self.block_offsets, self.codes, None,
                            self.block_init, self.flags, int(self.codes.numel()) - N.MH_CODES_PAD)

    def tables(self, prepare_lut: bool = True, stream: Optional[torch.cuda.Stream] = None):
        """T1/T2 (+ prepared table) built on the device from the device header."""
        from .decoder import DeviceTables
        return DeviceTables.from_canonical_header(self.canon, self.canon.device, prepare_lut, stream)

    def result(self) -> DeviceEncodedFrame:
        st, n = int(self.status.item()), int(self.codes_len.item())
        N.check(st, "mh_encode_frame_device_async")
        return DeviceEncodedFrame(self.width, self.height, self.canon.cpu().numpy(), self.codes[:n],
                                  self.block_offsets, self.block_init, self.flags)


class BatchEncoder:
    """n_frames frames of one size per call (mh_encode_frames_device_async): each frame
    gets its own histogram, tree and codes (byte-identical to codec.encode_frame, frame
    by frame), in three launches whatever n_frames. Codes land in fixed 16-byte
    aligned slots of `slot` bytes (the capacity), so the result is one DeviceFrames
    batch for decode() when the frames share a table (e.g. block shuffles)."""

    def __init__(self, width: int, height: int, n_frames: int, device="cuda"):
        self.device = _dev(device)
        self.width, self.height, self.n = width, height, n_frames
        bw, bh = block_grid(width, height)
        self.nb = bw * bh
        ws = int(N.lib().mh_encode_frames_workspace_bytes(width, height, n_frames))
        # zero-filled once: every call leaves the histograms zeroed (MH_ENCODE_WORKSPACE_ZEROED)
        self.workspace = torch.zeros(ws + 256, dtype=torch.uint8, device=self.device)
        self.slot = (self.nb * 64 * 2 + N.MH_CODES_PAD + 15) // 16 * 16 + 16

    def encode_async(self, grays: torch.Tensor, flags: int = 0, init_zero_delta: bool = False,
                     stream: Optional[torch.cuda.Stream] = None) -> "AsyncEncodedBatch":
        """grays: contiguous uint8 [n, H, W] on the encoder's device, ready on `stream`."""
        if (grays.dtype != torch.uint8 or tuple(grays.shape) != (self.n, self.height, self.width)
                or not grays.is_contiguous()):
            raise ValueError(f"grays must be contiguous uint8 [{self.n}, {self.height}, {self.width}]")
        if grays.device != self.device:
            raise ValueError("grays must live on the encoder's device")
        n = self.n
        with torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext():
            codes = torch.empty(n * self.slot + 16, dtype=torch.uint8, device=self.device)
            offs = torch.empty(n * self.nb, dtype=torch.int32, device=self.device)
            init = torch.empty(n * self.nb, dtype=torch.uint8, device=self.device) if init_zero_delta else None
            canon = torch.empty((n, 256), dtype=torch.uint8, device=self.device)
            lens = torch.empty(n, dtype=torch.int64, device=self.device)
            fco = torch.empty(n + 1, dtype=torch.int64, device=self.device)
            status = torch.empty(n, dtype=torch.int32, device=self.device)
        cbase = (codes.data_ptr() + 15) // 16 * 16
        base = self.workspace.data_ptr()
        aligned = (base + 255) // 256 * 256
        N.check(N.lib().mh_encode_frames_device_async(
            grays.data_ptr(), self.height * self.width, n, self.width, self.height,
            flags | N.MH_ENCODE_WORKSPACE_ZEROED, canon.data_ptr(), cbase, self.slot, lens.data_ptr(),
            fco.data_ptr(), offs.data_ptr(), init.data_ptr() if init is not None else None, status.data_ptr(),
            aligned, self.workspace.numel() - (aligned - base), _stream_ptr(stream, self.device)),
            "mh_encode_frames_device_async")
        view = codes[cbase - codes.data_ptr(): cbase - codes.data_ptr() + n * self.slot]
        return AsyncEncodedBatch(self.width, self.height, n, self.slot, canon, view, lens, fco, status, offs,
                                 init, flags)


@dataclasses.dataclass
class AsyncEncodedBatch:
    """A batched encode in flight: everything on the device (per-frame slots).

    Host synchronisation: frames() synchronises the stream once by default (check=True,
    since round 5: it reads `status` and `codes_len`); a pipeline that overlaps encode with
    decode must call frames(check=False), which stays asynchronous, and check `status`
    itself. frame(f) always synchronises."""
    width: int
    height: int
    n_frames: int
    slot: int
    canon: torch.Tensor               # u8[n, 256]
    codes: torch.Tensor               # u8[n * slot]
    codes_len: torch.Tensor           # int64[n] (payload + MH_CODES_PAD; 0 on an error)
    frame_code_offsets: torch.Tensor  # int64[n + 1] = f * slot
    status: torch.Tensor              # int32[n]
    block_offsets: torch.Tensor       # int32 view of u32[n * NB]
    block_init: Optional[torch.Tensor]
    flags: int

    def frames(self, check: bool = True) -> DeviceFrames:
        """All slots as one DeviceFrames batch (valid when the frames share a table).

        check=True (default) synchronises once: it raises MHError if any frame was
        rejected (that frame's slot and block offsets were never written, so decoding
        the batch would read garbage), and `code_bytes` is the batch's payload bytes
        (sum of codes_len minus the pads), as for DeviceFrames.pack. check=False stays
        asynchronous: the caller must check `status` before trusting a decode of the
        batch, and `code_bytes` is then the slots' capacity (n * slot minus the pads),
        an upper bound of the payload."""
        if check:
            st = self.status.cpu()
            bad = [i for i in range(self.n_frames) if int(st[i])]
            if bad:
                raise N.MHError(int(st[bad[0]]), f"mh_encode_frames_device_async: frame(s) {bad[:8]} rejected")
            payload = int(self.codes_len.sum().item()) - self.n_frames * N.MH_CODES_PAD
        else:
            payload = int(self.codes.numel()) - self.n_frames * N.MH_CODES_PAD
        return DeviceFrames(self.width, self.height, self.n_frames, self.block_offsets, self.codes,
                            self.frame_code_offsets, self.block_init, self.flags, payload)

    def frame(self, f: int) -> DeviceEncodedFrame:
        """Frame f (synchronises; raises MHError on a rejected frame)."""
        st, n = int(self.status[f].item()), int(self.codes_len[f].item())
        N.check(st, "mh_encode_frames_device_async")
        nb = self.block_offsets.numel() // self.n_frames
        init = self.block_init[f * nb:(f + 1) * nb] if self.block_init is not None else None
        return DeviceEncodedFrame(self.width, self.height, self.canon[f].cpu().numpy(),
                                  self.codes[f * self.slot: f * self.slot + n],
                                  self.block_offsets[f * nb:(f + 1) * nb], init, self.flags)


def encode_frame_device(gray: torch.Tensor, flags: int = 0, init_zero_delta: bool = False) -> DeviceEncodedFrame:
    """One-shot GPU encode of a [H, W] uint8 device tensor."""
    h, w = gray.shape
    return Encoder(w, h, gray.device).encode(gray, flags, init_zero_delta)

"""Frames streamed from host memory (BASELINE config 5): a thin wrapper over the
native mh_stream_* API (csrc/mh_stream.cpp) -- per-slot device buffers, one HIP
stream and one captured decode graph per slot (copy then decode in stream order) -- mirroring the
reference's per-frame command buffer (Shared/AAPLRenderer.m:1178-1921)."""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np
import torch

from . import _native as N
from .decoder import DeviceTables, _dev


class FrameStream:
    def __init__(self, tables: DeviceTables, width: int, height: int, codes_capacity: int,
                 slots: int = 2, flags: int = 0, block_init: bool = False, device="cuda"):
        dev = _dev(device)
        self.device, self.width, self.height = dev, width, height
        self.pitch = (width + 7) // 8 * 8
        self.outputs = [torch.empty((height, self.pitch), dtype=torch.uint8, device=dev)
                        for _ in range(slots)]
        proto = N.mh_frame()
        proto.d_table1 = tables.table1.data_ptr()
        proto.d_table2 = tables.table2.data_ptr()
        proto.table2_entries = tables.table2_entries
        proto.d_lut = tables.lut.data_ptr() if tables.lut is not None else None
        proto.dims = N.mh_dims(width, height, (width + 7) // 8, (height + 7) // 8)
        proto.n_frames = 1
        proto.flags = flags
        self._init_dummy = torch.zeros(8, dtype=torch.uint8, device=dev) if block_init else None
        proto.d_block_init = self._init_dummy.data_ptr() if block_init else None
        outs = (ctypes.c_void_p * slots)(*[t.data_ptr() for t in self.outputs])
        self._tables = tables  # keep the tables alive with the graphs that read them
        self._h = ctypes.c_void_p()
        N.check(N.lib().mh_stream_create(ctypes.byref(proto), int(codes_capacity), slots,
                                         outs, ctypes.byref(self._h)), "mh_stream_create")

    def submit(self, codes: torch.Tensor, offsets: torch.Tensor,
               init: Optional[torch.Tensor] = None) -> int:
        """Queue one frame from host tensors (pinned for an asynchronous DMA):
        codes u8 (payload + MH_CODES_PAD zero bytes), offsets u32/int32[NB]."""
        slot = ctypes.c_uint32(0)
        N.check(N.lib().mh_stream_submit(self._h, codes.data_ptr(), codes.numel(), offsets.data_ptr(),
                                         init.data_ptr() if init is not None else None,
                                         ctypes.byref(slot)), "mh_stream_submit")
        return int(slot.value)

    def output(self, slot: int) -> torch.Tensor:
        """[H, pitch] raster of `slot` (valid until `slots` further submits)."""
        return self.outputs[slot]

    def slot_stream(self, slot: int) -> int:
        """hipStream_t of `slot` (its copy and decode run there, in order)."""
        return int(N.lib().mh_stream_slot_stream(self._h, slot) or 0)

    def wait(self, slot: int) -> None:
        N.check(N.lib().mh_stream_wait(self._h, slot), "mh_stream_wait")

    def slot_time_ms(self, slot: int) -> float:
        """Device time of that slot's last frame: H2D copy start -> decode end."""
        ms = ctypes.c_float(0)
        N.check(N.lib().mh_stream_slot_time(self._h, slot, ctypes.byref(ms)), "mh_stream_slot_time")
        return float(ms.value)

    def synchronize(self) -> None:
        N.check(N.lib().mh_stream_synchronize(self._h), "mh_stream_synchronize")

    def close(self) -> None:
        if self._h:
            N.check(N.lib().mh_stream_destroy(self._h), "mh_stream_destroy")
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class FrameStreamGroup:
    """Frames round-robined over several devices (config 5 on N GPUs): one native
    stream per member (mh_stream_group_*), member i on devices[i] with its own copy
    of the tables; frame k goes to member k mod n. `tables` holds one DeviceTables
    per member, each resident on that member's device (a device may repeat)."""

    def __init__(self, tables, width: int, height: int, codes_capacity: int, slots: int = 2,
                 flags: int = 0):
        self.width, self.height = width, height
        self.pitch = (width + 7) // 8 * 8
        n = len(tables)
        protos = (N.mh_frame * n)()
        devs = (ctypes.c_int * n)()
        for i, t in enumerate(tables):
            p = protos[i]
            p.d_table1 = t.table1.data_ptr()
            p.d_table2 = t.table2.data_ptr()
            p.table2_entries = t.table2_entries
            p.d_lut = t.lut.data_ptr() if t.lut is not None else None
            p.dims = N.mh_dims(width, height, (width + 7) // 8, (height + 7) // 8)
            p.n_frames = 1
            p.flags = flags
            devs[i] = t.table1.device.index or 0
        self.devices = [int(d) for d in devs]
        self._tables = list(tables)
        self._h = ctypes.c_void_p()
        N.check(N.lib().mh_stream_group_create(protos, n, devs, int(codes_capacity), slots,
                                               ctypes.byref(self._h)), "mh_stream_group_create")
        self.size = int(N.lib().mh_stream_group_size(self._h))

    def submit(self, codes: torch.Tensor, offsets: torch.Tensor) -> tuple[int, int]:
        """Queue one frame from pinned host tensors -> (member, slot)."""
        m, slot = ctypes.c_uint32(0), ctypes.c_uint32(0)
        N.check(N.lib().mh_stream_group_submit(self._h, codes.data_ptr(), codes.numel(), offsets.data_ptr(),
                                               None, ctypes.byref(m), ctypes.byref(slot)),
                "mh_stream_group_submit")
        return int(m.value), int(slot.value)

    def _member(self, member: int):
        h = N.lib().mh_stream_group_member(self._h, member)
        if not h:
            raise IndexError(member)
        return h

    def output(self, member: int, slot: int) -> torch.Tensor:
        """[H, pitch] raster of (member, slot) on that member's device (a view of the
        stream's own buffer; valid until `slots` further submits to that member)."""
        pitch = ctypes.c_size_t(0)
        ptr = N.lib().mh_stream_output(self._member(member), slot, ctypes.byref(pitch))
        dev = torch.device("cuda", self.devices[member])
        return _device_view(ptr, (self.height, int(pitch.value)), dev)

    def wait(self, member: int, slot: int) -> None:
        N.check(N.lib().mh_stream_wait(self._member(member), slot), "mh_stream_wait")

    def slot_time_ms(self, member: int, slot: int) -> float:
        """Device time of that slot's last frame: H2D copy start -> decode end."""
        ms = ctypes.c_float(0)
        N.check(N.lib().mh_stream_slot_time(self._member(member), slot, ctypes.byref(ms)), "mh_stream_slot_time")
        return float(ms.value)

    def synchronize(self) -> None:
        N.check(N.lib().mh_stream_group_synchronize(self._h), "mh_stream_group_synchronize")

    def close(self) -> None:
        if self._h:
            N.check(N.lib().mh_stream_group_destroy(self._h), "mh_stream_group_destroy")
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _device_view(ptr: int, shape, device: torch.device) -> torch.Tensor:
    """A uint8 tensor over device memory the library owns (no copy, no ownership)."""
    n = int(np.prod(shape))

    class _Arr:
        __cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (int(ptr), False),
                                    "version": 3, "strides": None}
    with torch.cuda.device(device):
        return torch.as_tensor(_Arr(), device=device).view(*shape)


def pinned_frame(ef) -> tuple[torch.Tensor, torch.Tensor]:
    """Host-pinned (codes, block offsets) of an EncodedFrame, laid out in one buffer
    as the stream's slots are ([offsets, padded to 16 B][codes]) so a submit is one DMA."""
    offs = np.ascontiguousarray(ef.block_offsets, np.uint32)
    ob = (offs.size * 4 + 15) // 16 * 16
    buf = torch.zeros(ob + ef.codes.size, dtype=torch.uint8).pin_memory()
    buf[: offs.size * 4].copy_(torch.from_numpy(offs.view(np.uint8)))
    buf[ob:].copy_(torch.from_numpy(np.ascontiguousarray(ef.codes)))
    return buf[ob:], buf[: offs.size * 4].view(torch.int32)

"""ctypes binding of libmetalhuffman_amd.so (the C-ABI in include/metalhuffman.h).

The library is loaded from this package directory only. If it is missing the
import fails loudly: there is no CPU fallback for the decode path.
"""
from __future__ import annotations

import ctypes
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MH_LIB") or os.path.join(_PKG, "libmetalhuffman_amd.so")

MH_OK = 0
MH_FLAG_NO_DELTA = 0x1
MH_FLAG_LANE_PAIRS = 0x2  # lane-pair single-frame decode: diagnostic library only (diag_lanepairs())
MH_FLAG_ANY_ORDER = 0x4  # the launch may overlap earlier work on the stream (caller guarantees independence)
MH_ENCODE_WORKSPACE_ZEROED = 0x100  # the encoder workspace was zero-filled once (mh_encode_frame_device*)
MH_CODES_PAD = 4
MH_TABLE2_MAX_ENTRIES = 257 * 256
MH_MAX_DIM = 65535

# every symbol include/metalhuffman.h declares
EXPORTS = (
    "mh_decode", "mh_lut_bytes", "mh_prepare_lut", "mh_lut_bits", "mh_split_blocks",
    "mh_merge_blocks", "mh_encode_signed_byte_deltas", "mh_decode_signed_byte_deltas",
    "mh_codes_bound", "mh_encode_huffman", "mh_encode_frame", "mh_canonical_codes",
    "mh_build_tables", "mh_build_single_table", "mh_error_string", "mh_device_count",
    "mh_build_tables_device", "mh_stream_create", "mh_stream_submit", "mh_stream_output",
    "mh_stream_compute_stream", "mh_stream_slot_stream", "mh_stream_wait", "mh_stream_synchronize",
    "mh_stream_destroy", "mh_stream_slot_time", "mh_stream_device",
    "mh_stream_group_create", "mh_stream_group_submit", "mh_stream_group_member", "mh_stream_group_size",
    "mh_stream_group_synchronize", "mh_stream_group_destroy",
    "mh_code_lengths", "mh_encode_workspace_bytes", "mh_encode_frame_device",
    "mh_encode_frame_device_async", "mh_encode_frames_workspace_bytes", "mh_encode_frames_device_async",
    "mh_container_header", "mh_parse_container_header", "mh_check",
    "mh_decode_huffman_bits", "mh_decode_huffman_bits_from_tables", "mh_decode_frame_cpu",
    "mh_build_stamp",
)


class MHError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        msg = lib().mh_error_string(status).decode() if _lib is not None else str(status)
        super().__init__(f"{what}: {msg} (status {status})" if what else f"{msg} (status {status})")


class mh_dims(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint32), ("height", ctypes.c_uint32),
                ("block_width", ctypes.c_uint32), ("block_height", ctypes.c_uint32)]


class mh_frame(ctypes.Structure):
    _fields_ = [
        ("d_block_offsets", ctypes.c_void_p),
        ("d_codes", ctypes.c_void_p),
        ("codes_bytes", ctypes.c_uint64),
        ("d_frame_code_offsets", ctypes.c_void_p),
        ("d_table1", ctypes.c_void_p),
        ("d_table2", ctypes.c_void_p),
        ("table2_entries", ctypes.c_uint32),
        ("d_lut", ctypes.c_void_p),
        ("d_block_init", ctypes.c_void_p),
        ("dims", mh_dims),
        ("n_frames", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
    ]


_lib = None

_vp = ctypes.c_void_p
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u16p = ctypes.POINTER(ctypes.c_uint16)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)


_diag_lp = None


def diag_lanepairs() -> ctypes.CDLL:
    """The lane-pair diagnostic library (metalhuffman_amd/diag/libmh_diag_lanepairs.so,
    built by `python -m metalhuffman_amd.build`): north_star's lane-group cursor, a
    measured negative kept for A/B and its parity tests. It exports
    one entry point, mh_diag_decode_lanepairs, with mh_decode's signature; the product
    library refuses MH_FLAG_LANE_PAIRS."""
    global _diag_lp
    if _diag_lp is None:
        from . import build as _build
        path = _build.diag_lib_path("lanepairs")
        if not os.path.exists(path):
            raise ImportError(f"{path} not found: build it with `python -m metalhuffman_amd.build`")
        L = ctypes.CDLL(path)
        L.mh_build_stamp.restype = ctypes.c_char_p
        want, have = "diag:lanepairs:" + _build.diag_stamp("lanepairs"), L.mh_build_stamp().decode()
        if have != want:
            raise ImportError(f"{path} was built from other sources: rebuild with `python -m metalhuffman_amd.build`")
        L.mh_diag_decode_lanepairs.argtypes = [ctypes.POINTER(mh_frame), _vp, ctypes.c_size_t, ctypes.c_size_t,
                                               _vp]
        _diag_lp = L
    return _diag_lp


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} not found: build it with `python -m metalhuffman_amd.build` "
                "(the HIP decoder has no fallback)")
        L = ctypes.CDLL(LIB_PATH)
        L.mh_build_stamp.restype = ctypes.c_char_p
        if not os.environ.get("MH_LIB"):  # experiment variants (MH_LIB) carry extra -D flags
            from . import build as _build

            want, have = _build.library_stamp(), L.mh_build_stamp().decode()
            if have != want:
                raise ImportError(
                    f"{LIB_PATH} was built from other sources (stamp {have[:16]}, sources {want[:16]}): "
                    "rebuild with `python -m metalhuffman_amd.build`")
        L.mh_decode.argtypes = [ctypes.POINTER(mh_frame), _vp, ctypes.c_size_t, ctypes.c_size_t, _vp]
        L.mh_check.argtypes = [ctypes.POINTER(mh_frame), _vp, _vp]
        L.mh_lut_bytes.restype = ctypes.c_size_t
        L.mh_lut_bits.restype = ctypes.c_int
        L.mh_prepare_lut.argtypes = [_vp, _vp, ctypes.c_uint32, _vp, _vp]
        L.mh_build_tables_device.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp, _vp]
        L.mh_stream_create.argtypes = [ctypes.POINTER(mh_frame), ctypes.c_uint64, ctypes.c_uint32,
                                       ctypes.POINTER(_vp), ctypes.POINTER(_vp)]
        L.mh_stream_submit.argtypes = [_vp, _vp, ctypes.c_uint64, _vp, _vp, _u32p]
        L.mh_stream_output.argtypes = [_vp, ctypes.c_uint32, ctypes.POINTER(ctypes.c_size_t)]
        L.mh_stream_output.restype = _vp
        L.mh_stream_compute_stream.argtypes = [_vp]
        L.mh_stream_compute_stream.restype = _vp
        L.mh_stream_slot_stream.argtypes = [_vp, ctypes.c_uint32]
        L.mh_stream_slot_stream.restype = _vp
        L.mh_stream_wait.argtypes = [_vp, ctypes.c_uint32]
        L.mh_stream_synchronize.argtypes = [_vp]
        L.mh_stream_destroy.argtypes = [_vp]
        L.mh_stream_slot_time.argtypes = [_vp, ctypes.c_uint32, ctypes.POINTER(ctypes.c_float)]
        L.mh_stream_device.argtypes = [_vp]
        L.mh_stream_group_create.argtypes = [ctypes.POINTER(mh_frame), ctypes.c_uint32,
                                             ctypes.POINTER(ctypes.c_int), ctypes.c_uint64, ctypes.c_uint32,
                                             ctypes.POINTER(_vp)]
        L.mh_stream_group_submit.argtypes = [_vp, _vp, ctypes.c_uint64, _vp, _vp, _u32p, _u32p]
        L.mh_stream_group_member.argtypes = [_vp, ctypes.c_uint32]
        L.mh_stream_group_member.restype = _vp
        L.mh_stream_group_size.argtypes = [_vp]
        L.mh_stream_group_size.restype = ctypes.c_uint32
        L.mh_stream_group_synchronize.argtypes = [_vp]
        L.mh_stream_group_destroy.argtypes = [_vp]
        L.mh_code_lengths.argtypes = [_u64p, _u8p]
        L.mh_container_header.argtypes = [ctypes.c_uint64, _u8p]
        L.mh_parse_container_header.argtypes = [_u8p, _u64p]
        L.mh_encode_workspace_bytes.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        L.mh_encode_workspace_bytes.restype = ctypes.c_size_t
        L.mh_encode_frame_device.argtypes = [_vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _u8p,
                                             _vp, ctypes.c_uint64, _u64p, _vp, _vp, _vp, ctypes.c_size_t,
                                             _vp]
        L.mh_encode_frame_device_async.argtypes = [_vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                   _vp, _vp, ctypes.c_uint64, _vp, _vp, _vp, _vp, _vp,
                                                   ctypes.c_size_t, _vp]
        L.mh_encode_frames_workspace_bytes.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
        L.mh_encode_frames_workspace_bytes.restype = ctypes.c_size_t
        L.mh_encode_frames_device_async.argtypes = [_vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                                    ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, ctypes.c_uint64,
                                                    _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_size_t, _vp]
        L.mh_split_blocks.argtypes = [_u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_uint8, _u8p, ctypes.c_size_t]
        L.mh_merge_blocks.argtypes = [_u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _u8p,
                                      ctypes.c_size_t]
        L.mh_encode_signed_byte_deltas.argtypes = [_u8p, _u8p, ctypes.c_size_t]
        L.mh_decode_signed_byte_deltas.argtypes = [_u8p, _u8p, ctypes.c_size_t]
        L.mh_codes_bound.argtypes = [ctypes.c_uint64]
        L.mh_codes_bound.restype = ctypes.c_uint64
        L.mh_encode_huffman.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_uint32, _u8p, _u8p,
                                        ctypes.c_uint64, _u64p, _u32p]
        L.mh_encode_frame.argtypes = [_u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _u8p,
                                      _u8p, ctypes.c_uint64, _u64p, _u32p, _u8p]
        L.mh_canonical_codes.argtypes = [_u8p, _u16p]
        L.mh_build_tables.argtypes = [_u8p, _u8p, _u8p, ctypes.c_uint32, _u32p]
        L.mh_build_single_table.argtypes = [_u8p, _u8p]
        L.mh_decode_huffman_bits.argtypes = [_u8p, ctypes.c_uint64, _u8p, ctypes.c_uint64, _u8p, _u32p]
        L.mh_decode_huffman_bits_from_tables.argtypes = [_u8p, _u8p, ctypes.c_uint32, ctypes.c_uint32,
                                                         ctypes.c_uint32, ctypes.c_uint64, _u8p,
                                                         ctypes.c_uint64, _u8p, _u32p]
        L.mh_decode_frame_cpu.argtypes = [_u32p, _u8p, ctypes.c_uint64, _u8p, _u8p, ctypes.c_uint32, _u8p,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _u8p,
                                          ctypes.c_size_t, ctypes.c_uint32]
        L.mh_error_string.argtypes = [ctypes.c_int]
        L.mh_error_string.restype = ctypes.c_char_p
        L.mh_device_count.restype = ctypes.c_int
        _lib = L
    return _lib


def check(status: int, what: str = "") -> None:
    if status != MH_OK:
        raise MHError(status, what)

"""TEST INFRASTRUCTURE ONLY -- ctypes binding of the plain-C oracle (mh_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module. It restates mdejong/MetalHuffman's CPU codec (Shared/HuffmanEncoder.cpp,
Shared/HuffmanUtil.cpp, Shared/huff_util.hpp, Util.m's block split) and the Metal
decode semantics (Shared/AAPLShaders.metal); see mh_oracle.h for per-function
file:line citations.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import tempfile

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libmh_oracle.so")
REF_ENCODE = os.path.join(_HERE, "_ref", "ref_encode")

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u16p = ctypes.POINTER(ctypes.c_uint16)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def build_ref() -> bool:
    """Compile the reference encoder from /root/reference (container only)."""
    if not os.path.isdir("/root/reference/Shared"):
        return False
    subprocess.run(["make", "-s", "-C", _HERE, "ref"], check=True)
    return os.path.exists(REF_ENCODE)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_split_blocks.argtypes = [_u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint8, _u8p]
        L.orc_delta_encode.argtypes = [_u8p, ctypes.c_size_t]
        L.orc_delta_decode.argtypes = [_u8p, ctypes.c_size_t]
        L.orc_code_lengths.argtypes = [_u8p, ctypes.c_uint32, _u8p]
        L.orc_canonical_codes.argtypes = [_u8p, _u16p]
        L.orc_huffman_encode.argtypes = [_u8p, ctypes.c_uint32, ctypes.c_uint32, _u8p, _u8p,
                                         ctypes.c_uint64, _u64p, _u32p]
        L.orc_split_tables.argtypes = [_u8p, _u8p, _u8p, ctypes.c_uint32, _u32p]
        L.orc_single_table.argtypes = [_u8p, _u8p]
        L.orc_decode_from_tables.argtypes = [_u8p, _u8p, ctypes.c_uint32, _u8p, _u8p, _u32p]
        L.orc_decode_single_table.argtypes = [_u8p, ctypes.c_uint32, _u8p, _u8p, _u32p]
        L.orc_decode_frame_shader.argtypes = [_u32p, _u8p, _u8p, _u8p, ctypes.c_uint32,
                                              ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                              _u8p, ctypes.c_int, _u8p]
        L.orc_encode_frame.argtypes = [_u8p, ctypes.c_uint32, ctypes.c_uint32, _u8p, _u8p,
                                       ctypes.c_uint64, _u64p, _u32p]
        L.orc_time_decode_frames.argtypes = [_u8p, _u8p, ctypes.c_uint32,
                                             ctypes.POINTER(_u8p), ctypes.POINTER(_u8p),
                                             ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
        L.orc_time_decode_frames.restype = ctypes.c_double
        L.orc_time_decode_pipeline.argtypes = [_u8p, _u8p, ctypes.c_uint32, ctypes.c_uint32,
                                               ctypes.POINTER(_u8p), ctypes.POINTER(_u8p),
                                               ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
        L.orc_time_decode_pipeline.restype = ctypes.c_double
        L.orc_check_frame.argtypes = [_u32p, _u8p, ctypes.c_uint64, _u8p, _u8p, ctypes.c_uint32,
                                      ctypes.c_uint32, _u32p]
        _lib = L
    return _lib


def _p(a: np.ndarray, t=_u8p):
    return a.ctypes.data_as(t)


class OracleError(RuntimeError):
    pass


def _check(rc: int, what: str):
    if rc != 0:
        raise OracleError(f"{what} failed rc={rc}")


def split_blocks(img: np.ndarray, bdim: int = 8, zero: int = 0) -> np.ndarray:
    h, w = img.shape
    bw, bh = -(-w // bdim), -(-h // bdim)
    img = np.ascontiguousarray(img, dtype=np.uint8)
    out = np.empty(bw * bh * bdim * bdim, np.uint8)
    _check(lib().orc_split_blocks(_p(img), w, h, bdim, bw, bh, zero, _p(out)), "split")
    return out


def delta_encode(buf: np.ndarray) -> np.ndarray:
    b = np.array(buf, dtype=np.uint8, copy=True)
    lib().orc_delta_encode(_p(b), b.size)
    return b


def delta_decode(buf: np.ndarray) -> np.ndarray:
    b = np.array(buf, dtype=np.uint8, copy=True)
    lib().orc_delta_decode(_p(b), b.size)
    return b


def code_lengths(sym: np.ndarray) -> tuple[int, np.ndarray]:
    sym = np.ascontiguousarray(sym, dtype=np.uint8)
    canon = np.zeros(256, np.uint8)
    rc = lib().orc_code_lengths(_p(sym), sym.size, _p(canon))
    return rc, canon


def canonical_codes(canon: np.ndarray) -> np.ndarray:
    canon = np.ascontiguousarray(canon, dtype=np.uint8)
    codes = np.zeros(256, np.uint16)
    lib().orc_canonical_codes(_p(canon), _p(codes, _u16p))
    return codes


def huffman_encode(sym: np.ndarray, stride: int = 64):
    """-> canon[256], codes (encoder bytes incl. its 2 zero bytes), offsets u32."""
    sym = np.ascontiguousarray(sym, dtype=np.uint8)
    n = sym.size
    cap = 2 * n + 16
    canon = np.zeros(256, np.uint8)
    codes = np.zeros(cap, np.uint8)
    ln = ctypes.c_uint64(0)
    offs = np.zeros(max(1, n // stride), np.uint32)
    _check(lib().orc_huffman_encode(_p(sym), n, stride, _p(canon), _p(codes), cap,
                                    ctypes.byref(ln), _p(offs, _u32p)), "encode")
    return canon, codes[: ln.value].copy(), offs[: n // stride].copy()


def split_tables(canon: np.ndarray):
    canon = np.ascontiguousarray(canon, dtype=np.uint8)
    t1 = np.zeros(512, np.uint8)
    t2 = np.zeros(257 * 256 * 2, np.uint8)
    ent = ctypes.c_uint32(0)
    _check(lib().orc_split_tables(_p(canon), _p(t1), _p(t2), 257 * 256, ctypes.byref(ent)),
           "split_tables")
    return t1, t2[: 2 * ent.value].copy()


def single_table(canon: np.ndarray) -> np.ndarray:
    canon = np.ascontiguousarray(canon, dtype=np.uint8)
    t = np.zeros(65536 * 2, np.uint8)
    _check(lib().orc_single_table(_p(canon), _p(t)), "single_table")
    return t


def decode_from_tables(t1, t2, nsym: int, buf: np.ndarray, want_offsets=False):
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    out = np.zeros(nsym, np.uint8)
    offs = np.zeros(nsym, np.uint32) if want_offsets else None
    lib().orc_decode_from_tables(_p(t1), _p(t2), nsym, _p(buf), _p(out),
                                 _p(offs, _u32p) if want_offsets else None)
    return (out, offs) if want_offsets else out


def decode_single_table(t, nsym: int, buf: np.ndarray):
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    out = np.zeros(nsym, np.uint8)
    lib().orc_decode_single_table(_p(t), nsym, _p(buf), _p(out), None)
    return out


def decode_frame_shader(offsets, codes, t1, t2, w, h, block_init=None, delta=True):
    bw, bh = -(-w // 8), -(-h // 8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    out = np.zeros((h, w), np.uint8)
    bi = None
    if block_init is not None:
        bi = np.ascontiguousarray(block_init, dtype=np.uint8)
    _check(lib().orc_decode_frame_shader(_p(offsets, _u32p), _p(codes), _p(t1), _p(t2), w, h,
                                         bw, bh, _p(bi) if bi is not None else None,
                                         1 if delta else 0, _p(out)), "decode_frame_shader")
    return out


def check_frame(offsets, codes, t1, t2) -> np.ndarray:
    """Debug report of one frame (see orc_check_frame): u32[4]."""
    offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    t1 = np.ascontiguousarray(t1, dtype=np.uint8)
    t2 = np.ascontiguousarray(t2, dtype=np.uint8)
    rep = np.zeros(4, np.uint32)
    lib().orc_check_frame(_p(offsets, _u32p), _p(codes), ctypes.c_uint64(codes.size), _p(t1), _p(t2),
                          ctypes.c_uint32(t2.size // 2), ctypes.c_uint32(offsets.size), _p(rep, _u32p))
    return rep


def encode_frame(img: np.ndarray):
    """-> canon, huffBuff (codes + 4 zero pad bytes total), block offsets."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    nb = (-(-w // 8)) * (-(-h // 8))
    cap = nb * 64 * 2 + 16
    canon = np.zeros(256, np.uint8)
    codes = np.zeros(cap, np.uint8)
    offs = np.zeros(nb, np.uint32)
    ln = ctypes.c_uint64(0)
    _check(lib().orc_encode_frame(_p(img), w, h, _p(canon), _p(codes), cap, ctypes.byref(ln),
                                  _p(offs, _u32p)), "encode_frame")
    return canon, codes[: ln.value].copy(), offs


def time_decode_frames(t1, t2, nsym: int, bufs: list, n_threads: int, reps: int = 1) -> float:
    n = len(bufs)
    outs = [np.zeros(nsym, np.uint8) for _ in range(n)]
    BA = _u8p * n
    b_arr = BA(*[_p(b) for b in bufs])
    o_arr = BA(*[_p(o) for o in outs])
    return lib().orc_time_decode_frames(_p(t1), _p(t2), nsym, b_arr, o_arr, n, n_threads, reps)


def time_decode_pipeline(t1, t2, w: int, h: int, bufs: list, n_threads: int, reps: int = 1,
                         rasters: list | None = None) -> float:
    """Wall seconds to decode + undelta + raster `bufs` (frame-parallel on n_threads),
    repeated `reps` times. `rasters` (optional) receives the last pass's W x H frames."""
    n = len(bufs)
    outs = rasters if rasters is not None else [np.zeros((h, w), np.uint8) for _ in range(n)]
    BA = _u8p * n
    b_arr = BA(*[_p(b) for b in bufs])
    o_arr = BA(*[_p(o) for o in outs])
    return lib().orc_time_decode_pipeline(_p(t1), _p(t2), w, h, b_arr, o_arr, n, n_threads, reps)


def ref_encode(sym: np.ndarray, stride: int = 64, with_header: bool = False):
    """Run the REAL reference encoder (oracle/_ref/ref_encode). Container only.
    -> canon, codes, offsets (+ the 8-byte container header with with_header)."""
    if not os.path.exists(REF_ENCODE):
        raise FileNotFoundError(REF_ENCODE)
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "in.bin")
        np.ascontiguousarray(sym, dtype=np.uint8).tofile(src)
        pre = os.path.join(d, "out")
        subprocess.run([REF_ENCODE, src, str(stride), pre], check=True,
                       stdout=subprocess.DEVNULL)
        canon = np.fromfile(pre + ".canon", np.uint8)
        codes = np.fromfile(pre + ".codes", np.uint8)
        offs = np.fromfile(pre + ".offsets", np.uint32)
        header = np.fromfile(pre + ".header", np.uint8)
    return (canon, codes, offs, header) if with_header else (canon, codes, offs)

"""The C-ABI boundary (include/metalhuffman.h): the library loads without a GPU,
exports every declared symbol, its struct layout matches the header, and the
decode entry points reject bad arguments before touching the device. CPU only."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "metalhuffman.h")


def _declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(mh_[a-z_0-9]+)\(", txt, re.M)))


def test_every_declared_symbol_is_exported(mh):
    names = _declared()
    assert len(names) >= 15
    lib = ctypes.CDLL(mh.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(mh.EXPORTS)


def test_struct_layout_matches_header(mh):
    from metalhuffman_amd import _native as N
    fields = [f for f, _ in N.mh_frame._fields_]
    src = "#include <stdio.h>\n#include <stddef.h>\n#include \"metalhuffman.h\"\nint main(void){\n"
    src += 'printf("%zu %zu\\n", sizeof(mh_frame), sizeof(mh_lookup_symbol));\n'
    for f in fields:
        src += f'printf("%zu\\n", offsetof(mh_frame, {f}));\n'
    src += "return 0;}\n"
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split()
    assert int(out[0]) == ctypes.sizeof(N.mh_frame)
    assert int(out[1]) == 2
    for f, off in zip(fields, out[2:]):
        assert getattr(N.mh_frame, f).offset == int(off), f


def _frame(**kw):
    from metalhuffman_amd import _native as N
    fr = N.mh_frame()
    fr.d_block_offsets = 0x10000
    fr.d_codes = 0x20000
    fr.codes_bytes = 4096
    fr.d_table1 = 0x30000
    fr.d_table2 = 0x40000
    fr.table2_entries = 256
    fr.dims = N.mh_dims(2048, 1536, 256, 192)
    fr.n_frames = 1
    for k, v in kw.items():
        setattr(fr, k, v)
    return fr


@pytest.mark.parametrize("kw,status", [
    (dict(d_codes=None), -1),
    (dict(flags=0x80), -1),
    (dict(flags=0x8), -1),                                     # first unassigned flag bit
    (dict(flags=0x2, codes_bytes=2), -4),                      # lane pairs: accepted (and ignored) by the product
    (dict(n_frames=0), -1),
    (dict(n_frames=2), -1),                                    # batch without frame offsets
    (dict(table2_entries=100), -5),
    (dict(table2_entries=258 * 256), -5),
    (dict(d_codes=0x20004), -6),                               # not 16-byte aligned
    (dict(codes_bytes=2), -4),
])
def test_decode_rejects_bad_frames(mh, kw, status):
    from metalhuffman_amd import _native as N
    fr = _frame(**kw)
    assert N.lib().mh_decode(ctypes.byref(fr), 0x50000, 2048, 0, None) == status


def test_decode_rejects_bad_dims_and_pitch(mh):
    from metalhuffman_amd import _native as N
    L = N.lib()
    assert L.mh_decode(None, 0x50000, 2048, 0, None) == -1
    assert L.mh_decode(ctypes.byref(_frame(dims=N.mh_dims(2048, 1536, 255, 192))), 0x50000, 2048, 0, None) == -2
    assert L.mh_decode(ctypes.byref(_frame(dims=N.mh_dims(70000, 8, 8750, 1))), 0x50000, 70000, 0, None) == -2
    assert L.mh_decode(ctypes.byref(_frame()), 0x50000, 2044, 0, None) == -6    # pitch % 8
    assert L.mh_decode(ctypes.byref(_frame()), 0x50000, 1024, 0, None) == -4    # pitch < width
    assert L.mh_prepare_lut(0x30000, 0x40000, 300, 0x60000, None) == -5
    assert L.mh_prepare_lut(None, 0x40000, 256, 0x60000, None) == -1
    assert L.mh_build_tables_device(None, 0x30000, 0x40000, 0x50000, None, None, None) == -1
    assert L.mh_build_tables_device(0x10000, 0x30000, 0x40000, 0x50000, 0x60004, None, None) == -6
    h = ctypes.c_void_p()
    assert L.mh_stream_create(None, 4096, 2, None, ctypes.byref(h)) == -1
    assert L.mh_stream_create(ctypes.byref(_frame()), 4096, 0, None, ctypes.byref(h)) == -1
    assert L.mh_stream_create(ctypes.byref(_frame(dims=N.mh_dims(16, 16, 3, 2))), 4096, 2, None,
                              ctypes.byref(h)) == -2
    assert L.mh_stream_submit(None, 0x1000, 4096, 0x2000, None, None) == -1
    n = ctypes.c_uint64()
    canon = (ctypes.c_uint8 * 256)()
    assert L.mh_encode_frame_device(None, 8, 8, 0, canon, 0x1000, 64, ctypes.byref(n), 0x2000, None,
                                    0x10000, 1 << 20, None) == -1
    assert L.mh_encode_frame_device(0x100, 0, 8, 0, canon, 0x1000, 64, ctypes.byref(n), 0x2000, None,
                                    0x10000, 1 << 20, None) == -2
    assert L.mh_encode_frame_device(0x100, 8, 8, 0, canon, 0x1002, 64, ctypes.byref(n), 0x2000, None,
                                    0x10000, 1 << 20, None) == -6
    assert L.mh_encode_frame_device(0x100, 8, 8, 0, canon, 0x1000, 64, ctypes.byref(n), 0x2000, None,
                                    0x10000, 16, None) == -4
    assert L.mh_encode_workspace_bytes(2048, 1536) >= 49152 * 64
    ws = L.mh_encode_workspace_bytes(64, 64)
    assert L.mh_encode_frame_device_async(None, 8, 8, 0, 0x3000, 0x1000, 64, None, 0x2000, None, None,
                                          0x10000, ws, None) == -1
    assert L.mh_encode_frame_device_async(0x100, 8, 8, 2, 0x3000, 0x1000, 64, None, 0x2000, None, None,
                                          0x10000, ws, None) == -1
    assert L.mh_encode_frame_device_async(0x100, 8, 70000, 0, 0x3000, 0x1000, 64, None, 0x2000, None,
                                          None, 0x10000, ws, None) == -2
    assert L.mh_encode_frame_device_async(0x100, 8, 8, 0, 0x3000, 0x1000, 64, None, 0x2000, None, None,
                                          0x10080, ws, None) == -6
    assert L.mh_encode_frame_device_async(0x100, 64, 64, 0, 0x3000, 0x1000, 64, None, 0x2000, None,
                                          None, 0x10000, 256, None) == -4
    assert L.mh_check(None, 0x70000, None) == -1
    assert L.mh_check(ctypes.byref(_frame()), None, None) == -1
    assert L.mh_check(ctypes.byref(_frame(n_frames=2)), 0x70000, None) == -1
    assert L.mh_check(ctypes.byref(_frame(dims=N.mh_dims(2048, 1536, 255, 192))), 0x70000, None) == -2
    assert L.mh_check(ctypes.byref(_frame(table2_entries=100)), 0x70000, None) == -5
    assert L.mh_check(ctypes.byref(_frame()), 0x70002, None) == -6


def test_lane_pair_kernel_only_in_diagnostic_library(mh):
    """the lane-pair kernel (a measured negative kept for A/B) is not
    in the product library; the diagnostic library carries it behind its one entry point,
    which validates like mh_decode and accepts MH_FLAG_LANE_PAIRS."""
    import metalhuffman_amd.build as B
    from metalhuffman_amd import _native as N
    B.build_diag()
    prod = subprocess.run(["nm", "-D", "--defined-only", mh.LIB_PATH], check=True, capture_output=True,
                          text=True).stdout
    assert "lanepair" not in prod and "lanepair" not in open(mh.LIB_PATH, "rb").read().decode("latin-1")
    diag = B.diag_lib_path("lanepairs")
    syms = subprocess.run(["nm", "-D", "--defined-only", diag], check=True, capture_output=True,
                          text=True).stdout
    exported = sorted(l.split()[-1] for l in syms.splitlines() if " T " in l)
    assert exported == ["mh_build_stamp", "mh_diag_decode_lanepairs"], exported
    assert "lanepair_kernel" in open(diag, "rb").read().decode("latin-1")
    L = N.diag_lanepairs()
    assert L.mh_diag_decode_lanepairs(ctypes.byref(_frame(flags=0x8)), 0x50000, 2048, 0, None) == -1
    assert L.mh_diag_decode_lanepairs(ctypes.byref(_frame(codes_bytes=2, flags=0x2)), 0x50000, 2048, 0,
                                      None) == -4


def test_constants(mh):
    from metalhuffman_amd import _native as N
    L = N.lib()
    assert L.mh_lut_bits() == 13
    assert L.mh_lut_bytes() % 16 == 0 and L.mh_lut_bytes() >= 2 * 8192
    assert L.mh_codes_bound(100) >= 100 * 2
    assert L.mh_error_string(-3) == b"huffman code longer than 16 bits"


def test_stream_group_argument_checks():
    """mh_stream_group_*: argument validation happens before any HIP call."""
    import ctypes
    import metalhuffman_amd as mh
    from metalhuffman_amd import _native as N
    L = mh.lib()
    h = ctypes.c_void_p()
    devs = (ctypes.c_int * 1)(0)
    protos = (N.mh_frame * 1)()
    assert L.mh_stream_group_create(None, 1, devs, 4096, 2, ctypes.byref(h)) == -1
    assert L.mh_stream_group_create(protos, 0, devs, 4096, 2, ctypes.byref(h)) == -1
    assert L.mh_stream_group_create(protos, 1, None, 4096, 2, ctypes.byref(h)) == -1
    assert L.mh_stream_group_submit(None, None, 0, None, None, None, None) == -1
    assert L.mh_stream_group_size(None) == 0
    assert not L.mh_stream_group_member(None, 0)
    assert L.mh_stream_group_synchronize(None) == -1
    assert L.mh_stream_group_destroy(None) == -1
    f = ctypes.c_float()
    assert L.mh_stream_slot_time(None, 0, ctypes.byref(f)) == -1
    assert L.mh_stream_device(None) == -1

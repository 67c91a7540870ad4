"""The product library's gfx950 code objects (CPU only): no kernel spills registers or
uses scratch. Round 5 found a batch-kernel variant that spilled (80 VGPRs + 40 B of
scratch, a flavour branch taken with the first span in flight) and decoded the flat
8192^2 frame wrongly on the GPU; the kernels' register budget is part of their design
(DESIGN.md section 4), so a spill is a build failure, not a slow path."""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import tempfile

import pytest

LLVM = "/opt/rocm/lib/llvm/bin"


def _kernels(lib_path):
    objdump, readelf = os.path.join(LLVM, "llvm-objdump"), os.path.join(LLVM, "llvm-readelf")
    if not (os.path.exists(objdump) and os.path.exists(readelf)):
        pytest.skip("ROCm llvm tools not found")
    out = {}
    with tempfile.TemporaryDirectory() as d:
        lib = os.path.join(d, os.path.basename(lib_path))
        shutil.copy(lib_path, lib)
        subprocess.run([objdump, "--offloading", lib], cwd=d, check=True, capture_output=True)
        cos = [f for f in os.listdir(d) if "amdgcn-amd-amdhsa--gfx950" in f]
        assert cos, os.listdir(d)
        for co in cos:
            notes = subprocess.run([readelf, "--notes", os.path.join(d, co)], check=True, capture_output=True,
                                   text=True).stdout
            for blk in re.split(r"\n\s+- \.", notes):
                m = re.search(r"\.name:\s+(\S+)", blk)
                if not m or "kernel" not in m.group(1):
                    continue
                get = lambda k: int(re.search(rf"\.{k}:\s+(\d+)", blk).group(1))
                out[m.group(1)] = (get("private_segment_fixed_size"), get("vgpr_spill_count"),
                                   get("sgpr_spill_count"), get("vgpr_count"))
    return out


def test_product_kernels_do_not_spill(mh):
    ks = _kernels(mh.LIB_PATH)
    names = " ".join(ks)
    for k in ("mh_decode_kernel", "mh_decode_small_kernel", "enc_pack_wave_kernel", "enc_split_kernel",
              "mh_build_tables_kernel"):
        assert k in names, k
    bad = {k: v for k, v in ks.items() if v[0] or v[1] or v[2]}
    assert not bad, bad
    # the batch kernel's occupancy budget: 6 waves per SIMD (3 x 8-wave workgroups per CU)
    for k, v in ks.items():
        if "mh_decode_kernel" in k:
            assert v[3] <= 80, (k, v)

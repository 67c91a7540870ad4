"""The product library's gfx950 code objects (CPU only).

1. No 64-bit VALU shift (v_lshlrev_b64 / v_lshrrev_b64 / v_ashrrev_i64) takes its shift
   amount from the last VGPR of its kernel's allocation (index 8k+7 with the next VGPR
   unallocated). That is the cause of round 5's silent miscompute (DESIGN.md section 4,
   "Round 5's miscompute"): a batch-kernel build with 80 VGPRs put one shift amount in
   v79 and decoded that symbol wrongly in ~0.5 % of tiles on the GPU; the same code object
   with only that amount moved to another VGPR decoded every tile right, and an s_nop in
   front did not help (profiles/r06_forensic_isa_patch.txt). LLVM guards this pattern for
   gfx90a only (GCNHazardRecognizer::fixShift64HighRegBug), so nothing in hipcc's gfx950
   output rules it out: this test does.
2. No kernel spills registers or uses scratch: the kernels' register budget is part of
   their design, so a spill is a build failure, not a slow path.
   (Round 5's failing build also spilled; a spill is what filled v79 there.)"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import tempfile

import pytest

LLVM = "/opt/rocm/lib/llvm/bin"


_SHIFT64 = re.compile(r"\b(v_lshlrev_b64|v_lshrrev_b64|v_ashrrev_i64)(?:_e64)?\s+v\[\d+:\d+\],\s*v(\d+)\b")


def high_reg_shifts(disasm: str, vgpr_count: dict) -> list:
    """(kernel, instruction) pairs whose 64-bit shift amount is the last VGPR of the kernel's
    8-register allocation granule with the next VGPR unallocated (vgpr_count: kernel symbol
    -> .vgpr_count; functions not in it are skipped)."""
    bad, cur, alloc = [], None, 0
    for line in disasm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = m.group(1)
            n = vgpr_count.get(cur)
            alloc = (n + 7) // 8 * 8 if n is not None else 0
            continue
        if cur is None or not alloc:
            continue
        m = _SHIFT64.search(line)
        if m:
            r = int(m.group(2))
            if r % 8 == 7 and r + 1 >= alloc:
                bad.append((cur, line.strip()))
    return bad


def test_high_reg_shift_checker():
    """The checker flags exactly round 5's pattern (amount in v79 of an 80-VGPR kernel)."""
    text = ("0000000000001000 <k80>:\n"
            "  v_lshrrev_b64 v[68:69], v79, v[50:51]  // 000000001000: D2910044 0002654F\n"
            "  v_lshrrev_b64 v[68:69], v78, v[50:51]\n"
            "0000000000002000 <k88>:\n"
            "  v_lshrrev_b64 v[68:69], v79, v[50:51]\n"
            "0000000000003000 <k72>:\n"
            "  v_lshlrev_b64 v[2:3], v71, v[4:5]\n  v_ashrrev_i64 v[2:3], v63, v[4:5]\n")
    bad = high_reg_shifts(text, {"k80": 80, "k88": 88, "k72": 72})
    assert [b[0] for b in bad] == ["k80", "k72"], bad


def _disasm(lib_path):
    objdump = os.path.join(LLVM, "llvm-objdump")
    if not os.path.exists(objdump):
        pytest.skip("ROCm llvm tools not found")
    with tempfile.TemporaryDirectory() as d:
        lib = os.path.join(d, os.path.basename(lib_path))
        shutil.copy(lib_path, lib)
        subprocess.run([objdump, "--offloading", lib], cwd=d, check=True, capture_output=True)
        cos = [f for f in os.listdir(d) if "amdgcn-amd-amdhsa--gfx950" in f]
        assert cos, os.listdir(d)
        return "\n".join(subprocess.run([objdump, "-d", "--mcpu=gfx950", os.path.join(d, co)], check=True,
                                        capture_output=True, text=True).stdout for co in cos)


def test_no_shift_amount_in_last_vgpr(mh):
    ks = _kernels(mh.LIB_PATH)
    text = _disasm(mh.LIB_PATH)
    assert "v_lshrrev_b64" in text
    bad = high_reg_shifts(text, {k: v[3] for k, v in ks.items()})
    assert not bad, bad[:8]


def test_diagnostic_libraries_no_shift_amount_in_last_vgpr(mh):
    """The same guard on the diagnostic libraries the GPU tests load (lane pairs, spin-0)."""
    import metalhuffman_amd.build as B
    B.build_diag()
    for name in B.DIAG_LIBS:
        path = B.diag_lib_path(name)
        ks = _kernels(path)
        bad = high_reg_shifts(_disasm(path), {k: v[3] for k, v in ks.items()})
        assert not bad, (name, bad[:8])


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

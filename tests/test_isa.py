"""The product library's gfx950 code objects (CPU only).

1. No 64-bit VALU shift (v_lshlrev_b64 / v_lshrrev_b64 / v_ashrrev_i64) takes its shift
   amount from the last VGPR of its kernel's allocation (index 8k+7 with the next VGPR
   unallocated). That is the cause of round 5's silent miscompute (DESIGN.md section 4,
   "Round 5's miscompute"): a batch-kernel build with 80 VGPRs put one shift amount in
   v79 and decoded that symbol wrongly in ~0.5 % of tiles on the GPU; the same code object
   with only that amount moved to another VGPR decoded every tile right, and an s_nop in
   front did not help (profiles/r06_forensic_isa_patch.txt). LLVM guards this pattern for
   gfx90a only (GCNHazardRecognizer::fixShift64HighRegBug), so nothing in hipcc's gfx950
   output rules it out: this test does, and build() runs the same check (metalhuffman_amd/isa_guard.py)
   before it installs a library.
2. No kernel spills registers or uses scratch: the kernels' register budget is part of
   their design, so a spill is a build failure, not a slow path.
   (Round 5's failing build also spilled; a spill is what filled v79 there.)"""
from __future__ import annotations

import pytest

from metalhuffman_amd.isa_guard import check_library, high_reg_shifts


def _tools():
    from metalhuffman_amd import isa_guard
    if not isa_guard.available():
        pytest.skip("ROCm llvm tools not found")
    return isa_guard


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
    return _tools().disasm(lib_path)


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
    return _tools().kernels(lib_path)


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


def test_build_guard_passes_product_and_diag(mh):
    """The check build() runs before installing a library finds nothing in the shipped ones."""
    import metalhuffman_amd.build as B
    _tools()
    for path in [mh.LIB_PATH] + B.build_diag():
        assert check_library(path) == [], path

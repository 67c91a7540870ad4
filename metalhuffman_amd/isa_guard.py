"""Build-time check of the gfx950 code objects in a linked library (CPU only, no GPU).

build() runs it on every library it links and refuses to install one that fails, so a
compiler or source change cannot ship the pattern behind round 5's silent miscompute
("Round 5's miscompute"):
1. a 64-bit VALU shift (v_lshlrev_b64 / v_lshrrev_b64 / v_ashrrev_i64) whose shift amount is
   the last VGPR of its kernel's allocation (index 8k+7 with the next VGPR unallocated).
   On gfx950 such a shift gave wrong results intermittently; the same code object with only
   that amount moved to another VGPR decoded every tile right
   (profiles/r06_forensic_isa_patch.txt). LLVM guards the pattern for gfx90a only
   (GCNHazardRecognizer::fixShift64HighRegBug), so nothing in hipcc's gfx950 output rules it out;
2. a kernel with register spills or scratch: the kernels' register budget is part of their
   design, and round 5's failing build spilled (a spill filled v79).
tests/test_isa.py applies the same checks to the product and diagnostic libraries.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import tempfile

LLVM = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "llvm", "bin")
OBJDUMP = os.path.join(LLVM, "llvm-objdump")
READELF = os.path.join(LLVM, "llvm-readelf")

_SHIFT64 = re.compile(r"\b(v_lshlrev_b64|v_lshrrev_b64|v_ashrrev_i64)(?:_e64)?\s+v\[\d+:\d+\],\s*v(\d+)\b")


def available() -> bool:
    return os.path.exists(OBJDUMP) and os.path.exists(READELF)


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


def _code_objects(lib_path: str, d: str) -> list:
    lib = os.path.join(d, os.path.basename(lib_path))
    shutil.copy(lib_path, lib)
    subprocess.run([OBJDUMP, "--offloading", lib], cwd=d, check=True, capture_output=True)
    cos = [os.path.join(d, f) for f in os.listdir(d) if "amdgcn-amd-amdhsa--gfx950" in f]
    if not cos:
        raise RuntimeError(f"no gfx950 code object in {lib_path}")
    return cos


def disasm(lib_path: str) -> str:
    with tempfile.TemporaryDirectory() as d:
        return "\n".join(subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", co], check=True, capture_output=True,
                                        text=True).stdout for co in _code_objects(lib_path, d))


def kernels(lib_path: str) -> dict:
    """kernel symbol -> (private_segment_fixed_size, vgpr_spill_count, sgpr_spill_count,
    vgpr_count), from the code objects' metadata notes."""
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for co in _code_objects(lib_path, d):
            notes = subprocess.run([READELF, "--notes", co], check=True, capture_output=True, text=True).stdout
            for blk in re.split(r"\n\s+- \.", notes):
                m = re.search(r"\.name:\s+(\S+)", blk)
                if not m or "kernel" not in m.group(1):
                    continue
                get = lambda k: int(re.search(rf"\.{k}:\s+(\d+)", blk).group(1))
                out[m.group(1)] = (get("private_segment_fixed_size"), get("vgpr_spill_count"),
                                   get("sgpr_spill_count"), get("vgpr_count"))
    return out


def check_library(lib_path: str) -> list:
    """Problems found in a linked library (empty: it passes)."""
    ks = kernels(lib_path)
    problems = [f"{k}: scratch {v[0]} B, VGPR spills {v[1]}, SGPR spills {v[2]}"
                for k, v in ks.items() if v[0] or v[1] or v[2]]
    problems += [f"{k}: 64-bit shift amount in the last allocated VGPR: {ins}"
                 for k, ins in high_reg_shifts(disasm(lib_path), {k: v[3] for k, v in ks.items()})]
    return problems

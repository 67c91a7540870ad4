"""Build libmetalhuffman_amd.so in-tree (hipcc for gfx950 + g++ for the host codec).

    python -m metalhuffman_amd.build            # incremental
    python -m metalhuffman_amd.build --force

The shared library lands next to this file so it travels with the repository
snapshot to the GPU box; nothing is installed into site-packages.
"""
from __future__ import annotations

import argparse
import hashlib
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(PKG, "_build")
LIB = os.path.join(PKG, "libmetalhuffman_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("MH_OFFLOAD_ARCH", "gfx950")

SOURCES = {
    # kernarg preload: the decode kernels' leading scalar arguments arrive in SGPRs at wave
    # launch, so their first loads need no scalar load of the kernarg segment
    "mh_decode.o": ("mh_decode.hip", [HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
                                      "-Wall", "-mllvm", "-amdgpu-kernarg-preload-count=16", "-c"]),
    "mh_tables.o": ("mh_tables.hip", [HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
                                      "-Wall", "-c"]),
    "mh_encode.o": ("mh_encode.hip", [HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
                                      "-Wall", "-c"]),
    "mh_check.o": ("mh_check.hip", [HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
                                    "-Wall", "-c"]),
    "mh_stream.o": ("mh_stream.cpp", [HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
                                      "-Wall", "-c"]),
    "mh_host.o": ("mh_host.cpp", ["g++", "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wextra", "-c"]),
    "mh_cpu.o": ("mh_cpu.cpp", ["g++", "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wextra", "-pthread", "-c"]),
}
HEADERS = [os.path.join(ROOT, "include", "metalhuffman.h"), os.path.join(CSRC, "mh_lut.hpp")]
LINK_FLAGS = [f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread"]


def _sha(*parts) -> str:
    h = hashlib.sha256()
    for p in parts:
        h.update(p if isinstance(p, bytes) else str(p).encode())
        h.update(b"\0")
    return h.hexdigest()


def _read(path: str) -> bytes:
    with open(path, "rb") as f:
        return f.read()


def object_stamp(obj: str) -> str:
    """Content stamp of one object: its compile flags, its source and every header
    it can include. No path enters it, so the stamp is the same here and in the
    snapshot on the GPU box."""
    src, cmd = SOURCES[obj]
    return _sha(" ".join(cmd[1:]), src, _read(os.path.join(CSRC, src)), *[_read(h) for h in HEADERS])


def library_stamp() -> str:
    """The stamp compiled into libmetalhuffman_amd.so (mh_build_stamp())."""
    return _sha(*[object_stamp(o) for o in sorted(SOURCES)], " ".join(LINK_FLAGS))


def source_stamps() -> dict:
    """sha256[:16] of each product source plus the library stamp[:16]: printed by
    smoke() and carried in the bench line, so records tie numbers to sources."""
    out = {src: hashlib.sha256(_read(os.path.join(CSRC, src))).hexdigest()[:16] for src, _ in SOURCES.values()}
    out["lib"] = library_stamp()[:16]
    return out


def _stamp_ok(target: str, stamp: str) -> bool:
    try:
        return os.path.exists(target) and _read(target + ".stamp").decode().strip() == stamp
    except OSError:
        return False


def _write_stamp(target: str, stamp: str) -> None:
    with open(target + ".stamp", "w") as f:
        f.write(stamp + "\n")


def _stale(target: str, deps: list[str]) -> bool:
    """mtime rule, kept only for test-infrastructure programs (host demo, probes)."""
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def ensure_objects(force: bool = False, verbose: bool = False, only=None) -> list[str]:
    """Compile every default object (or those in `only`) whose content stamp is missing
    or stale, whatever the library's stamp says; returns the objects' paths. The
    diagnostic libraries link these objects, and _build/ does not travel to the GPU box,
    so they must not assume build() left them behind (it returns early on a current
    library)."""
    os.makedirs(BUILD, exist_ok=True)
    objs = []
    for obj, (src, cmd) in SOURCES.items():
        obj_path = os.path.join(BUILD, obj)
        objs.append(obj_path)
        if only is not None and obj not in only:
            continue
        st = object_stamp(obj)
        if force or not _stamp_ok(obj_path, st):
            full = cmd + [os.path.join(CSRC, src), "-o", obj_path]
            if verbose:
                print(" ".join(full), flush=True)
            subprocess.run(full, check=True)
            _write_stamp(obj_path, st)
    return objs


def _guard(lib: str) -> None:
    """Refuse to install a library whose code objects fail isa_guard.check_library (a 64-bit
    shift amount in a kernel's last VGPR -- round 5's miscompute -- or a spill)."""
    from . import isa_guard
    if not isa_guard.available():
        print(f"warning: {isa_guard.LLVM} missing, ISA guard skipped for {lib}", file=sys.stderr)
        return
    problems = isa_guard.check_library(lib)
    if problems:
        raise RuntimeError(f"ISA guard refused {lib} (left in place for inspection):\n  " + "\n  ".join(problems))


def build(force: bool = False, verbose: bool = False) -> str:
    """Rebuild by CONTENT, not mtime (a snapshot may carry any mtimes), and link the
    library with its stamp compiled in, so the loader can refuse a stale one.

    A library whose stamp equals the tree's (every source, header and flag) is
    current: nothing is compiled or linked. That is the GPU box's case -- the library
    is built here, in the build container, and travels with the snapshot (objects in
    _build/ do not); the box only checks the stamp, and _native.lib() refuses to load
    a library whose compiled-in stamp differs from the tree's sources."""
    lst = library_stamp()
    if not force and _stamp_ok(LIB, lst):
        return LIB
    objs = ensure_objects(force=force, verbose=verbose)
    if force or not _stamp_ok(LIB, lst):
        stamp_c = os.path.join(BUILD, "mh_stamp.c")
        with open(stamp_c, "w") as f:
            f.write("/* generated by metalhuffman_amd/build.py */\n"
                    f'const char* mh_build_stamp(void) {{ return "{lst}"; }}\n')
        stamp_o = os.path.join(BUILD, "mh_stamp.o")
        subprocess.run(["gcc", "-O2", "-fPIC", "-c", stamp_c, "-o", stamp_o], check=True)
        tmp = LIB + ".tmp"
        full = [HIPCC, *LINK_FLAGS, "-o", tmp] + objs + [stamp_o]
        if verbose:
            print(" ".join(full), flush=True)
        subprocess.run(full, check=True)
        _guard(tmp)
        os.replace(tmp, LIB)  # never rewrite a mapped library in place
        _write_stamp(LIB, lst)
    return LIB


DIAG_DIR = os.path.join(PKG, "diag")
# Diagnostic libraries: name -> (-D flags, the objects they change, standalone).
#   not standalone: the default library with some objects rebuilt, loaded INSTEAD of it
#     (MH_LIB) in a child process by the GPU tests;
#   standalone: only the changed objects (+ a stamp), loaded BESIDE the product library
#     (_native.diag_lanepairs()). The lane-pair kernel (MH_FLAG_LANE_PAIRS, a measured
#     negative kept for A/B) lives only there: the product library does not carry it.
DIAG_LIBS = {
    "spin0": (["MH_DIAG_SPIN_TICKS=0"], ["mh_encode.o"], False),  # encoder packers time out at once
    "lanepairs": (["MH_LANE_PAIRS=1"], ["mh_decode.o"], True),    # exports mh_diag_decode_lanepairs
}


def diag_lib_path(name: str) -> str:
    return os.path.join(DIAG_DIR, f"libmh_diag_{name}.so")


def diag_stamp(name: str) -> str:
    """The stamp compiled into a diagnostic library (after "diag:<name>:")."""
    defines = DIAG_LIBS[name][0]
    return _sha("diag", name, *defines, library_stamp())


def build_diag(force: bool = False, verbose: bool = False) -> list[str]:
    """The diagnostic libraries (content-stamped like the default one)."""
    build(verbose=verbose)
    os.makedirs(DIAG_DIR, exist_ok=True)
    out = []
    for name, (defines, changed, standalone) in DIAG_LIBS.items():
        lib = diag_lib_path(name)
        stamp = diag_stamp(name)
        out.append(lib)
        if not force and _stamp_ok(lib, stamp):
            continue
        tmpdir = os.path.join(BUILD, f"diag_{name}")
        os.makedirs(tmpdir, exist_ok=True)
        if not standalone:
            ensure_objects(verbose=verbose, only=[o for o in SOURCES if o not in changed])
        objs = []
        for obj, (src, cmd) in SOURCES.items():
            if standalone and obj not in changed:
                continue
            if obj in changed:
                o = os.path.join(tmpdir, obj)
                full = cmd + [f"-D{d}" for d in defines] + [os.path.join(CSRC, src), "-o", o]
                if verbose:
                    print(" ".join(full), flush=True)
                subprocess.run(full, check=True)
                objs.append(o)
            else:
                objs.append(os.path.join(BUILD, obj))
        stamp_c = os.path.join(tmpdir, "mh_stamp.c")
        with open(stamp_c, "w") as f:
            f.write(f'const char* mh_build_stamp(void) {{ return "diag:{name}:{stamp}"; }}\n')
        subprocess.run(["gcc", "-O2", "-fPIC", "-c", stamp_c, "-o", stamp_c[:-1] + "o"], check=True)
        subprocess.run([HIPCC, *LINK_FLAGS, "-o", lib + ".tmp"] + objs + [stamp_c[:-1] + "o"], check=True)
        _guard(lib + ".tmp")
        os.replace(lib + ".tmp", lib)
        _write_stamp(lib, stamp)
    return out


VARIANTS_DIR = os.path.join(ROOT, "ab")  # A/B libraries only; delete after an A/B session


def build_variant(name: str, defines: list[str], verbose: bool = False,
                  decode_src: str | None = None, src_override: dict | None = None) -> str:
    """Experiment builds (A/B on the GPU): same sources (or another mh_decode.hip, or
    any source replaced through src_override {name: path}), extra -D flags, loaded
    with MH_LIB=<path>. Never the default library."""
    over = dict(src_override or {})
    if decode_src:
        over["mh_decode.hip"] = decode_src
    os.makedirs(VARIANTS_DIR, exist_ok=True)
    tmp = os.path.join(BUILD, f"variant_{name}")
    os.makedirs(tmp, exist_ok=True)
    objs = []
    for obj, (src, cmd) in SOURCES.items():
        o = os.path.join(tmp, obj)
        path = over.get(src, os.path.join(CSRC, src))
        subprocess.run(cmd + [f"-D{d}" for d in defines] + [f"-I{CSRC}", path, "-o", o], check=True)
        objs.append(o)
    stamp_c = os.path.join(tmp, "mh_stamp.c")
    with open(stamp_c, "w") as f:
        f.write(f'const char* mh_build_stamp(void) {{ return "variant:{name}:{library_stamp()}"; }}\n')
    subprocess.run(["gcc", "-O2", "-fPIC", "-c", stamp_c, "-o", stamp_c[:-1] + "o"], check=True)
    out = os.path.join(VARIANTS_DIR, f"lib_{name}.so")
    subprocess.run([HIPCC, *LINK_FLAGS, "-o", out] + objs + [stamp_c[:-1] + "o"], check=True)
    if verbose:
        print(out)
    return out


HOST_SRC = os.path.join(ROOT, "host", "mh_decode_host.c")
HOST_BIN = os.path.join(ROOT, "host", "mh_decode_host")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def build_host(force: bool = False, verbose: bool = False) -> str:
    """The plain-C host program (host/mh_decode_host.c): gcc against the C-ABI
    header, libmetalhuffman_amd.so and the HIP runtime's C API."""
    lib = build(force=force, verbose=verbose)
    if force or _stale(HOST_BIN, [HOST_SRC, lib] + HEADERS):
        cmd = ["gcc", "-O2", "-std=c11", "-Wall", "-Wextra", "-D__HIP_PLATFORM_AMD__",
               "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROCM, "include"), HOST_SRC,
               "-o", HOST_BIN, "-L", PKG, "-lmetalhuffman_amd", "-L", os.path.join(ROCM, "lib"),
               "-lamdhip64", f"-Wl,-rpath,$ORIGIN/../metalhuffman_amd:{os.path.join(ROCM, 'lib')}"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return HOST_BIN


MULTI_SRC = os.path.join(ROOT, "host", "mh_decode_multi.c")
MULTI_BIN = os.path.join(ROOT, "host", "mh_decode_multi")


def build_host_multi(force: bool = False, verbose: bool = False) -> str:
    """The plain-C multi-GPU host (host/mh_decode_multi.c): one thread per device,
    RCCL broadcast of the 256-byte canonical header, batched device encode and decode."""
    lib = build(force=force, verbose=verbose)
    if force or _stale(MULTI_BIN, [MULTI_SRC, lib] + HEADERS):
        cmd = ["gcc", "-O2", "-std=c11", "-Wall", "-Wextra", "-pthread", "-D__HIP_PLATFORM_AMD__",
               "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROCM, "include"), MULTI_SRC,
               "-o", MULTI_BIN, "-L", PKG, "-lmetalhuffman_amd", "-L", os.path.join(ROCM, "lib"),
               "-lrccl", "-lamdhip64", f"-Wl,-rpath,$ORIGIN/../metalhuffman_amd:{os.path.join(ROCM, 'lib')}"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return MULTI_BIN


PROBE_SRC = os.path.join(ROOT, "scripts", "micro", "hbm_probe.hip")
PROBE_LIB = os.path.join(ROOT, "scripts", "micro", "libhbm_probe.so")
GATE_SRC = os.path.join(ROOT, "scripts", "micro", "launch_gate.hip")
GATE_LIB = os.path.join(ROOT, "scripts", "micro", "liblaunch_gate.so")


def build_probe(force: bool = False, verbose: bool = False) -> str:
    """bench.py's measurement infrastructure (not the decoder): the achievable-HBM
    probe reported beside the roofline (scripts/micro/libhbm_probe.so) and the
    timed-region launch gate (scripts/micro/liblaunch_gate.so)."""
    for src, lib in ((PROBE_SRC, PROBE_LIB), (GATE_SRC, GATE_LIB)):
        if force or _stale(lib, [src]):
            cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-shared", "-o", lib, src]
            if verbose:
                print(" ".join(cmd), flush=True)
            subprocess.run(cmd, check=True)
    return PROBE_LIB


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    args = ap.parse_args(argv)
    print(build(force=args.force, verbose=True))
    print(build_diag(force=args.force, verbose=True))
    print(build_host(force=args.force, verbose=True))
    print(build_host_multi(force=args.force, verbose=True))
    print(build_probe(force=args.force, verbose=True))
    return 0


if __name__ == "__main__":
    sys.exit(main())

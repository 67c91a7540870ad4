"""Build libmetalhuffman_amd.so in-tree (hipcc for gfx950 + g++ for the host codec).

    python -m metalhuffman_amd.build            # incremental
    python -m metalhuffman_amd.build --force

The shared library lands next to this file so it travels with the repository
snapshot to the GPU box; nothing is installed into site-packages.
"""
from __future__ import annotations

import argparse
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
    "mh_decode.o": ("mh_decode.hip", [HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
                                      "-Wall", "-c"]),
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


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    objs = []
    for obj, (src, cmd) in SOURCES.items():
        src_path = os.path.join(CSRC, src)
        obj_path = os.path.join(BUILD, obj)
        objs.append(obj_path)
        if force or _stale(obj_path, [src_path] + HEADERS):
            full = cmd + [src_path, "-o", obj_path]
            if verbose:
                print(" ".join(full), flush=True)
            subprocess.run(full, check=True)
    if force or _stale(LIB, objs):
        full = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", "-o", LIB] + objs
        if verbose:
            print(" ".join(full), flush=True)
        subprocess.run(full, check=True)
    return LIB


VARIANTS_DIR = os.path.join(PKG, "_variants")


def build_variant(name: str, defines: list[str], verbose: bool = False,
                  decode_src: str | None = None) -> str:
    """Experiment builds (A/B on the GPU): same sources (or another mh_decode.hip),
    extra -D flags, loaded with MH_LIB=<path>. Never the default library."""
    os.makedirs(VARIANTS_DIR, exist_ok=True)
    tmp = os.path.join(BUILD, f"variant_{name}")
    os.makedirs(tmp, exist_ok=True)
    objs = []
    for obj, (src, cmd) in SOURCES.items():
        o = os.path.join(tmp, obj)
        path = decode_src if (decode_src and src == "mh_decode.hip") else os.path.join(CSRC, src)
        subprocess.run(cmd + [f"-D{d}" for d in defines] + [f"-I{CSRC}", path, "-o", o], check=True)
        objs.append(o)
    out = os.path.join(VARIANTS_DIR, f"lib_{name}.so")
    subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", "-o", out] + objs, check=True)
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
    print(build_host(force=args.force, verbose=True))
    print(build_probe(force=args.force, verbose=True))
    return 0


if __name__ == "__main__":
    sys.exit(main())

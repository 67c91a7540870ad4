"""The host half of the C-ABI under the host compiler's AddressSanitizer and
UndefinedBehaviorSanitizer (CPU only; host code only -- the HIP kernels are not built).

host/mh_host_selftest.c links mh_host.cpp and mh_cpu.cpp (the producer and the CPU decoders)
and runs 135 cases: encode -> tables -> frame decode on 1 and 3 threads == the picture, the
producer's steps one by one through both serial CPU decoders (split tables and the single
64K table, HuffmanUtil.cpp:673-1046), the container header, and scrambled code bytes and
block offsets (memory safety only: the CPU frame decoder reads bytes past codes_bytes as
zero). Any sanitizer report aborts the program (-fno-sanitize-recover)."""
from __future__ import annotations

import os
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "metalhuffman_amd", "csrc")
SAN = ["-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"]


def test_host_codec_under_asan_ubsan():
    if not (shutil.which("gcc") and shutil.which("g++")):
        pytest.skip("host compilers not found")
    with tempfile.TemporaryDirectory() as d:
        objs = []
        for src, cc, std in (("mh_host.cpp", "g++", "-std=c++17"), ("mh_cpu.cpp", "g++", "-std=c++17")):
            o = os.path.join(d, src + ".o")
            subprocess.run([cc, *SAN, std, "-pthread", "-c", os.path.join(CSRC, src), "-o", o], check=True)
            objs.append(o)
        st = os.path.join(d, "selftest.o")
        subprocess.run(["gcc", *SAN, "-std=c11", "-Wall", "-Werror", "-c",
                        os.path.join(ROOT, "host", "mh_host_selftest.c"), "-o", st], check=True)
        exe = os.path.join(d, "selftest")
        subprocess.run(["g++", "-fsanitize=address,undefined", "-pthread", st, *objs, "-o", exe], check=True)
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
        for seed in ("1", "20261018"):
            r = subprocess.run([exe, seed], capture_output=True, text=True, env=env, timeout=300)
            assert r.returncode == 0 and "selftest ok 135" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])

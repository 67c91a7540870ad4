"""Stream-group bookkeeping on the CPU: metalhuffman_amd/csrc/mh_stream.cpp compiled
unchanged with g++ against fake HIP runtime calls (tests/stream_group_mock.cpp) that
track the current device. Checks the member round robin, each member's slot
rotation, that every copy/decode of a submit runs with the member's device current
and on that device's stream, that bad ordinals are refused, and that every
mh_stream_group_* call leaves the caller's device current (SURVEY.md 8(b)
threading; the reference's single queue: Shared/AAPLRenderer.m:996)."""
from __future__ import annotations

import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_stream_group_members_and_devices(tmp_path):
    exe = tmp_path / "stream_group_mock"
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
           os.path.join(ROOT, "tests", "stream_group_mock.cpp"),
           os.path.join(ROOT, "metalhuffman_amd", "csrc", "mh_stream.cpp"), "-o", str(exe)]
    subprocess.run(cmd, check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "failures 0" in r.stdout

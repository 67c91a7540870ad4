"""The plain-C host program (host/mh_decode_host.c) over the C-ABI: builds with gcc
against include/metalhuffman.h and, on the GPU, decodes bit-exactly -- including
buffers exactly as the reference encoder emitted them (golden.json)."""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

from helpers import golden


@pytest.fixture(scope="module")
def host_bin(mh):
    import metalhuffman_amd.build as B
    return B.build_host()


def _run(args, timeout=120):
    return subprocess.run(args, capture_output=True, text=True, timeout=timeout)


def test_host_builds_and_prints_usage(host_bin):
    r = _run([host_bin])
    assert r.returncode == 2 and "usage" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("wh", [(2048, 1536), (1001, 777), (8, 8), (13, 5)])
def test_host_synth(host_bin, wh):
    r = _run([host_bin, "synth", str(wh[0]), str(wh[1]), "5"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith(f"decode ok {wh[0]} {wh[1]} "), r.stdout
    assert " check 0 0 0 " in r.stdout  # mh_check: a clean stream


@pytest.mark.gpu
def test_host_raw_bigbridge(host_bin, bigbridge, tmp_path):
    p = tmp_path / "bb.gray"
    p.write_bytes(np.ascontiguousarray(bigbridge).tobytes())
    h, w = bigbridge.shape
    r = _run([host_bin, "raw", str(w), str(h), str(p), "20"])
    assert r.returncode == 0 and r.stdout.startswith(f"decode ok {w} {h} "), r.stdout + r.stderr


@pytest.mark.gpu
def test_host_reference_encoder_buffers(host_bin, tmp_path):
    """The reference encoder's own canonical header, codes and block offsets
    (golden.json) decoded unchanged by the C host."""
    n = 0
    for name, fx in golden()["small_frames"].items():
        w, h = fx["width"], fx["height"]
        canon = np.zeros(256, np.uint8)
        for k, v in fx["canon"].items():
            canon[int(k)] = v
        files = {"canon": canon.tobytes(), "codes": bytes.fromhex(fx["codes_hex"]),
                 "offsets": np.array(fx["block_offsets"], "<u4").tobytes(),
                 "expected": np.array(fx["pixels"], np.uint8).tobytes()}
        paths = []
        for k, v in files.items():
            p = tmp_path / f"{name}.{k}"
            p.write_bytes(v)
            paths.append(str(p))
        r = _run([host_bin, "buffers", str(w), str(h)] + paths)
        assert r.returncode == 0, (name, r.stdout, r.stderr)
        assert r.stdout.startswith(f"decode ok {w} {h} "), (name, r.stdout)
        n += 1
    assert n >= 5


@pytest.mark.gpu
@pytest.mark.parametrize("wh", [(2048, 1536), (1001, 777), (13, 5)])
def test_host_device_chain(host_bin, wh):
    """encode -> tables -> decode on the device through the C-ABI only: the device
    encoder's bytes equal the host codec's and the raster equals the frame."""
    r = _run([host_bin, "device", str(wh[0]), str(wh[1]), "5"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith(f"device ok {wh[0]} {wh[1]} "), r.stdout


def _multi_line(out: str) -> str:
    return next((ln for ln in out.splitlines() if ln.startswith(("multi ok", "FAIL"))), "")


@pytest.fixture(scope="module")
def multi_bin(mh):
    import metalhuffman_amd.build as B
    return B.build_host_multi()


def test_multi_host_builds_and_prints_usage(multi_bin):
    """The multi-GPU C host links against RCCL and the C-ABI (no GPU needed)."""
    r = _run([multi_bin])
    assert r.returncode == 2 and "usage" in r.stderr


@pytest.mark.gpu
def test_multi_host_rccl_world1(multi_bin, bigbridge, tmp_path):
    """host/mh_decode_multi at N = 1 on the box: RCCL
    communicator over the device, ncclBroadcast of device 0's 256-byte header, device
    table build, a 64-frame shard of BigBridge block shuffles encoded on the device in
    one batched call (every header equal to the broadcast one), batch decodes timed,
    every raster equal to its input. The same binary runs N = 2..8 on a full node."""
    p = tmp_path / "bb.gray"
    p.write_bytes(np.ascontiguousarray(bigbridge).tobytes())
    h, w = bigbridge.shape
    r = _run([multi_bin, "1", "64", "8", str(w), str(h), str(p)], timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    line = _multi_line(r.stdout)  # RCCL prints its version banner first
    assert line.startswith("multi ok 1 devices 64 frames_per_device 2048 1536"), r.stdout
    mbps = float(line.split("MBps_events ")[1].split()[0])
    assert mbps > 1e5, r.stdout  # a 64-frame launch decodes >> 1e5 MB/s on one MI355X
    # self-proving run: one line per device with its HIP ordinal and
    # PCI bus id, and the count of distinct devices that took part
    devs = [ln.split() for ln in r.stdout.splitlines() if ln.startswith("device ")]
    assert len(devs) == 1 and devs[0][2:4] == ["ordinal", "0"] and devs[0][4] == "pci", r.stdout
    assert devs[0][5].count(":") >= 2 and devs[0][-1] == "ok", r.stdout
    assert line.split()[-2:] == ["devices_verified", "1"], line


@pytest.mark.gpu
def test_multi_host_synthetic_small(multi_bin):
    r = _run([multi_bin, "1", "3", "2"], timeout=240)
    assert r.returncode == 0 and _multi_line(r.stdout).startswith("multi ok 1 devices 3 "), r.stdout + r.stderr

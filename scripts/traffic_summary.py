"""Per-launch HBM bytes of the decode kernels (mh_decode_kernel, mh_decode_small_kernel)
from rocprofv3 --pmc CSVs (gpu_traffic.sh).

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE/WRITE_SIZE are in
KiB; FETCH_SIZE reports half the bytes of wide coalesced streaming reads (x2);
WRITE_SIZE is exact for wide streaming stores.
"""
import csv
import glob
import json
import os
import statistics
import sys

root = sys.argv[1]
res = {}
kernels = {}
enc = {}
for d in sorted(glob.glob(os.path.join(root, "*_*_SIZE"))):
    base = os.path.basename(d)
    ctr = "FETCH_SIZE" if base.endswith("FETCH_SIZE") else "WRITE_SIZE"
    wl = base[: -len(ctr) - 1]
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            kn = r["Kernel_Name"]
            if r["Counter_Name"] != ctr:
                continue
            if wl == "encode":  # per kernel of the encoder
                for k in ("enc_split_kernel", "enc_code_kernel", "enc_one_kernel"):
                    if k in kn:
                        enc.setdefault(k, {}).setdefault(ctr, []).append(float(r["Counter_Value"]))
            elif "mh_decode_kernel" in kn or "mh_decode_small_kernel" in kn:
                vals.append(float(r["Counter_Value"]))
                kernels[wl] = "mh_decode_small_kernel" if "small" in kn else "mh_decode_kernel"
    if vals:
        res.setdefault(wl, {})[ctr] = statistics.median(vals) * 1024.0
        res[wl]["dispatches"] = len(vals)
out = {}
for wl, v in res.items():
    if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
        out[wl] = {"fetch_bytes_x2": round(2 * v["FETCH_SIZE"]), "write_bytes": round(v["WRITE_SIZE"]),
                   "traffic_bytes": round(2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]),
                   "dispatches": v["dispatches"], "kernel": kernels[wl]}
encode = {}
for k, v in enc.items():
    if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
        f, w = statistics.median(v["FETCH_SIZE"]) * 1024.0, statistics.median(v["WRITE_SIZE"]) * 1024.0
        encode[k] = {"fetch_bytes_x2": round(2 * f), "write_bytes": round(w), "traffic_bytes": round(2 * f + w),
                     "dispatches": len(v["FETCH_SIZE"])}
if encode:
    encode["frame"] = "2048x1536 BigBridge block shuffle (scripts/enc_profile.py)"
print(json.dumps({"per_launch_median": out, "encoder_per_launch_median": encode,
                  "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; FETCH x2 (gfx950)"},
                 indent=1))

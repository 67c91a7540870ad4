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
for d in sorted(glob.glob(os.path.join(root, "*_*_SIZE"))):
    base = os.path.basename(d)
    ctr = "FETCH_SIZE" if base.endswith("FETCH_SIZE") else "WRITE_SIZE"
    wl = base[: -len(ctr) - 1]
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            kn = r["Kernel_Name"]
            if ("mh_decode_kernel" in kn or "mh_decode_small_kernel" in kn) and r["Counter_Name"] == ctr:
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
print(json.dumps({"per_launch_median": out,
                  "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; FETCH x2 (gfx950)"},
                 indent=1))

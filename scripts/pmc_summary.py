"""Summarise rocprofv3 --pmc CSVs: per counter, mean per dispatch of one kernel."""
import csv, glob, sys, collections
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
pat = sys.argv[2] if len(sys.argv) > 2 else "mh_decode_kernel"
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0   # skip first N dispatches (warmup/parity)
vals = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/pmc*/run_counter_collection.csv")):
    rows = [r for r in csv.DictReader(open(f)) if pat in r["Kernel_Name"]]
    disp = sorted({int(r["Dispatch_Id"]) for r in rows})
    keep = set(disp[skip:])
    for r in rows:
        if int(r["Dispatch_Id"]) in keep:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(vals.items()):
    print(f"{k:28s} n={len(v):4d} mean={sum(v)/len(v):.4e} max={max(v):.4e}")

"""Per-dispatch PMC means of the batched encoder's kernels from rocprofv3 --pmc CSVs
(gpu_enc_batch.sh), and the HBM traffic per 64-frame call against the algorithmic
bytes (pixels in, codes + block offsets out).

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are
KiB; FETCH_SIZE reports half the bytes of wide coalesced streaming reads (x2).

    python scripts/enc_batch_pmc.py DIR [DIR ...] [--alg BYTES] [--calls N]

Values are per CALL (all of a call's dispatches of a kernel summed: a call may launch
each kernel once per sub-batch); enc_batch_profile.py 64 2 makes 7 calls.
"""
import csv
import glob
import os
import sys

args = sys.argv[1:]
alg = None
calls = 7
if "--calls" in args:
    i = args.index("--calls")
    calls = int(args[i + 1])
    del args[i:i + 2]
if "--alg" in args:
    i = args.index("--alg")
    alg = float(args[i + 1])
    del args[i:i + 2]
vals = {}
for d in args:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            kn = r["Kernel_Name"]
            for k in ("enc_split_kernel", "enc_tree_batch_kernel", "enc_pack_wave_kernel", "enc_pack_batch_kernel"):
                if k in kn:
                    vals.setdefault(k, {}).setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
                    vals[k][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
tot = {}
for k, cs in vals.items():
    print(f"== {k} (per call of the batch: sum over its dispatches)")
    for c, per in sorted(cs.items()):
        m = sum(per.values()) / calls
        print(f"  {c:24s} dispatches={len(per):3d} per_call={m:.4e}")
        if c in ("FETCH_SIZE", "WRITE_SIZE"):
            tot[c] = tot.get(c, 0.0) + m * 1024.0 * (2.0 if c == "FETCH_SIZE" else 1.0)
if tot:
    t = sum(tot.values())
    print(f"traffic per call: fetch {tot.get('FETCH_SIZE', 0) / 1e6:.1f} MB (x2 corrected), "
          f"write {tot.get('WRITE_SIZE', 0) / 1e6:.1f} MB, total {t / 1e6:.1f} MB"
          + (f", {t / alg:.3f} x algorithmic {alg / 1e6:.1f} MB" if alg else ""))

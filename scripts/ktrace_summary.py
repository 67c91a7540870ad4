"""Per-launch-shape durations of mh_decode_kernel from a rocprofv3 --kernel-trace CSV.

Grouped by kernel and launch shape; compare with the bench line's
roofline.kernel_us_avg of the same command (scripts/gpu_check.sh profiles one
workload per command). Counts include warm-up, the graph replay and the eager
per-launch pass, all the same launch.
"""
import collections
import csv
import glob
import statistics
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
groups = collections.defaultdict(list)
for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mh_decode" not in r["Kernel_Name"]:
            continue
        key = (r["Kernel_Name"].split("mh_decode")[1].split("_kernel")[0] or "batch", int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]), int(r["LDS_Block_Size"]), int(r["VGPR_Count"]))
        groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(f"{'kernel':>8} {'grid_threads':>12} {'wg':>5} {'lds':>6} {'vgpr':>5} {'n':>5} {'avg_us':>9} {'median_us':>9} {'min_us':>8}")
for (k, g, w, lds, v), d in sorted(groups.items(), key=lambda kv: -len(kv[1])):
    print(f"{k:>8} {g:12d} {w:5d} {lds:6d} {v:5d} {len(d):5d} {statistics.mean(d):9.3f} {statistics.median(d):9.3f} {min(d):8.3f}")

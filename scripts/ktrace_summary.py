"""Per-launch-shape durations of the decode kernels from a rocprofv3 --kernel-trace CSV.

Grouped by kernel and launch shape; compare with the bench line's
roofline.kernel_us_avg of the same command (scripts/gpu_check.sh profiles one
workload per command). `avg_us` is over every dispatch of the shape (warm-up, the
probe, untimed regions and the eager per-launch pass included). `timed_avg` and
`timed_span/K` (first start to last end, / K) are over the K dispatches of the timed
region whose HIP events give kernel_us_avg: bench.py brackets exactly that region with
two empty trace_marker_kernel launches (scripts/micro/launch_gate.hip), and the
decode dispatches between the last pair of markers are taken.

`timed_steady` = (end of the last of them - end of the first `unit`) / (K - unit): the
same back-to-back launch period as the line's kernel_us_avg (bench.roofline; `unit` =
the line's roofline.kernel_us_steady_unit: 1 for eager launches, 16 for long launches
replayed as 16-launch graphs).

    python scripts/ktrace_summary.py gpurun_out/prof_frame [K] [unit]
"""
import collections
import csv
import glob
import statistics
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
unit = int(sys.argv[3]) if len(sys.argv) > 3 else 1
groups = collections.defaultdict(list)
markers = []
for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "trace_marker_kernel" in r["Kernel_Name"]:
            markers.append(int(r["Start_Timestamp"]))
        if "mh_decode" not in r["Kernel_Name"]:
            continue
        key = (r["Kernel_Name"].split("mh_decode")[1].split("_kernel")[0] or "batch", int(r["Grid_Size_X"]),
               int(r["Workgroup_Size_X"]), int(r["LDS_Block_Size"]), int(r["VGPR_Count"]))
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        groups[key].append((s, e))


print(f"{'kernel':>8} {'grid_threads':>12} {'wg':>5} {'lds':>6} {'vgpr':>5} {'n':>5} {'avg_us':>9} "
      f"{'median_us':>9} {'min_us':>8} {'timed_avg':>9} {'timed_span/K':>12} {'timed_steady':>12}")
for (k, g, w, lds, v), d in sorted(groups.items(), key=lambda kv: -len(kv[1])):
    d.sort()
    dur = [(e - s) / 1e3 for s, e in d]
    n = len(dur)
    # the timed region: the decode dispatches between the last two trace markers
    timed = []
    if len(markers) >= 2:
        lo, hi = sorted(markers)[-2:]
        timed = [x for x in d if lo < x[0] < hi]
        timed = timed if len(timed) == steps else []
    ta = f"{statistics.mean((e - s) / 1e3 for s, e in timed):9.3f}" if timed else f"{'-':>9}"
    sp = f"{(timed[-1][1] - timed[0][0]) / 1e3 / len(timed):12.3f}" if timed else f"{'-':>12}"
    ok = timed and len(timed) > unit
    sd = f"{(timed[-1][1] - timed[unit - 1][1]) / 1e3 / (len(timed) - unit):12.3f}" if ok else f"{'-':>12}"
    print(f"{k:>8} {g:12d} {w:5d} {lds:6d} {v:5d} {n:5d} {statistics.mean(dur):9.3f} "
          f"{statistics.median(dur):9.3f} {min(dur):8.3f} {ta} {sp} {sd}")

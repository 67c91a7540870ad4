"""Per-launch-shape durations of the decode kernels from a rocprofv3 --kernel-trace CSV.

Grouped by kernel and launch shape; compare with the bench line's
roofline.kernel_us_avg of the same command (scripts/gpu_check.sh profiles one
workload per command). Counts include warm-up, the untimed first graph replay,
the timed graph replay and the eager per-launch pass (bench.Workload.run), all
the same launch. `timed_avg` (and timed_span/K, first start to last end / K) is over the timed region alone, K = --steps of
the profiled command (default 200): the K decode launches that follow the last
launch-gate kernel (bench.py's gated region, scripts/micro/launch_gate.hip), or, in a
trace without the gate, launches [n - 2K, n - K) in start order.

    python scripts/ktrace_summary.py gpurun_out/prof_frame [K]
"""
import collections
import csv
import glob
import statistics
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
groups = collections.defaultdict(list)
gates = []
for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gate_kernel" in r["Kernel_Name"]:
            gates.append(int(r["Start_Timestamp"]))
        if "mh_decode" not in r["Kernel_Name"]:
            continue
        key = (r["Kernel_Name"].split("mh_decode")[1].split("_kernel")[0] or "batch", int(r["Grid_Size_X"]),
               int(r["Workgroup_Size_X"]), int(r["LDS_Block_Size"]), int(r["VGPR_Count"]))
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        groups[key].append((s, e))


def runs_of(d, gap_ns=20000):
    """Back-to-back runs (next start within gap_ns of the previous end)."""
    out, cur = [], []
    for s, e in d:
        if cur and s - cur[-1][1] > gap_ns:
            out.append(cur)
            cur = []
        cur.append((s, e))
    if cur:
        out.append(cur)
    return out


print(f"{'kernel':>8} {'grid_threads':>12} {'wg':>5} {'lds':>6} {'vgpr':>5} {'n':>5} {'avg_us':>9} "
      f"{'median_us':>9} {'min_us':>8} {'timed_avg':>9} {'timed_span/K':>12}")
for (k, g, w, lds, v), d in sorted(groups.items(), key=lambda kv: -len(kv[1])):
    d.sort()
    dur = [(e - s) / 1e3 for s, e in d]
    n = len(dur)
    # the timed region: the K launches after the last launch gate (gated regions), or
    # else the run of K launches followed by exactly two more runs (bench.Workload.run:
    # timed replay, then the >=200-launch graph, then the eager per-launch pass)
    timed = []
    if gates:
        timed = [x for x in d if x[0] > max(gates)][:steps]
        timed = timed if len(timed) == steps else []
    else:
        rs = [r for r in runs_of(d) if len(r) >= steps]
        if len(rs) >= 3 and len(rs[-3]) == steps:
            timed = rs[-3]
    ta = f"{statistics.mean((e - s) / 1e3 for s, e in timed):9.3f}" if timed else f"{'-':>9}"
    sp = f"{(timed[-1][1] - timed[0][0]) / 1e3 / len(timed):12.3f}" if timed else f"{'-':>12}"
    print(f"{k:>8} {g:12d} {w:5d} {lds:6d} {v:5d} {n:5d} {statistics.mean(dur):9.3f} "
          f"{statistics.median(dur):9.3f} {min(dur):8.3f} {ta} {sp}")

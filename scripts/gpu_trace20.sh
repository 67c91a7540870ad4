# Kernel trace of the driver's 20-step bench command: per-launch durations in the timed replay.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof20
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof20 -o run -- python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/prof20.json 2> gpurun_out/prof20.err || { tail gpurun_out/prof20.err; exit 1; }
python3 - <<'PY'
import csv, glob
rows = list(csv.DictReader(open(glob.glob("gpurun_out/prof20/**/run_kernel_trace.csv", recursive=True)[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = [r for r in rows if "decode" in r["Kernel_Name"] or "gate" in r["Kernel_Name"]]
print(len(ks), "decode/gate launches")
prev_end = None
for r in ks[-70:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end else 0.0
    print(f"{r['Kernel_Name'][:40]:40s} dur {(e - s) / 1e3:7.2f} us  gap {gap:7.2f} us")
    prev_end = e
PY
cat gpurun_out/prof20.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('value', d['value'], 'ms', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'])"

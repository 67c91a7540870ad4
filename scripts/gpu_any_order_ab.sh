set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/ao.txt
for rep in 1 2; do
for ao in 0 1; do
  for st in 20 64; do
    r=$(MH_BENCH_ANY_ORDER=$ao timeout -k 10 300 python bench.py --workload frame --steps $st --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/ao.err) || { echo "ao=$ao FAILED"; tail gpurun_out/ao.err; exit 1; }
    echo "$r" | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('ao=$ao steps=$st value', d['value'], 'ms_per_step', d['ms_per_step'], 'region_us', d['roofline']['region_us_per_launch'], 'kernel_us', d['roofline']['kernel_us_avg'])" >> gpurun_out/ao.txt
  done
done
done
cat gpurun_out/ao.txt
rm -rf gpurun_out/prof_ao
MH_BENCH_ANY_ORDER=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_ao -o run -- python3 bench.py --workload frame --steps 64 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/ao_prof.json 2>gpurun_out/ao_prof.err || { tail gpurun_out/ao_prof.err; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_ao/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "small" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ov = sum(1 for a, b in zip(rows, rows[1:]) if int(b["Start_Timestamp"]) < int(a["End_Timestamp"]))
print("small-kernel dispatches", len(rows), "starting before the previous one ended:", ov)
gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(rows, rows[1:])]
gaps.sort()
print("start(n+1) - end(n) us: min %.2f p50 %.2f max %.2f" % (gaps[0], gaps[len(gaps)//2], gaps[-1]))
PY

# GPU round check: parity tests, smoke, bench, then rocprofv3 kernel traces of the
# bench command per workload (fail-fast).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log; grep -c PASSED gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
: > gpurun_out/ktrace_summary.txt
# same steps / warm-up as the bench line each number is compared with (the frame
# headline: 200 / 20; the extras: bench.py's own counts)
for spec in frame:20:5 batch:256:256 tile8192:512:512 tile8192_random:512:512; do
  IFS=: read wl k w <<< "$spec"
  rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_$wl
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$wl -o run -- python3 bench.py --workload $wl --steps $k --warmup $w --no-extras --no-cpu-baseline > gpurun_out/bench_prof_$wl.json 2> gpurun_out/bench_prof_$wl.err || { tail gpurun_out/bench_prof_$wl.err; exit 1; }
  u=$(python3 -c "import json;print(json.load(open('gpurun_out/bench_prof_$wl.json'))['roofline'].get('kernel_us_steady_unit') or 1)")
  { echo "== bench.py --workload $wl --steps $k --warmup $w (profiled line: roofline.kernel_us_avg $(python3 -c "import json;print(json.load(open('gpurun_out/bench_prof_$wl.json'))['roofline']['kernel_us_avg'])"), steady unit $u)"; python3 scripts/ktrace_summary.py gpurun_out/prof_$wl $k $u; } >> gpurun_out/ktrace_summary.txt
done
cat gpurun_out/ktrace_summary.txt
# producer side: the GPU encoder (async, back to back) and the device-only chain
rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_encode
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_encode -o run -- python3 scripts/enc_profile.py 64 > gpurun_out/enc_profile.log 2>&1 || { tail gpurun_out/enc_profile.log; exit 1; }
timeout -k 10 60 ./host/mh_decode_host device 2048 1536 200 > gpurun_out/device_chain.log 2>&1 || { cat gpurun_out/device_chain.log; exit 1; }
python3 - > gpurun_out/encoder_ktrace.txt <<'PY'
import csv
print([l for l in open("gpurun_out/enc_profile.log") if "async encode" in l][-1].strip())
print(open("gpurun_out/device_chain.log").read().strip())
for r in sorted(csv.DictReader(open("gpurun_out/prof_encode/run_kernel_stats.csv")), key=lambda r: -float(r["AverageNs"])):
    print(f"{float(r['AverageNs']) / 1e3:8.2f} us  x{r['Calls']:>4}  {r['Name'][:80]}")
PY
cat gpurun_out/encoder_ktrace.txt

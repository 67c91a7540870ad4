# Round-4 GPU check: a full rebuild on the box, parity tests, smoke, the driver's bench command, a rocprofv3 kernel
# trace of the headline workload, the batched encoder and the multi-GPU C host (fail-fast).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
# the library the tests load is compiled and linked HERE, on the box,
# from this snapshot's sources (--force: every object and the link), not the pushed one
sha256sum metalhuffman_amd/libmetalhuffman_amd.so > gpurun_out/build_on_box.log
timeout -k 10 900 python -m metalhuffman_amd.build --force >> gpurun_out/build_on_box.log 2>&1 || { tail -20 gpurun_out/build_on_box.log; exit 1; }
sha256sum metalhuffman_amd/libmetalhuffman_amd.so >> gpurun_out/build_on_box.log
grep -c -- "--offload-arch=gfx950" gpurun_out/build_on_box.log; tail -1 gpurun_out/build_on_box.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log; grep -c PASSED gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log | tail -1
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
rm -rf gpurun_out/prof_frame
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_frame -o run -- python3 bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/bench_prof_frame.json 2> gpurun_out/bench_prof_frame.err || { tail gpurun_out/bench_prof_frame.err; exit 1; }
{ echo "== bench.py --workload frame --steps 20 --warmup 5 (profiled line: roofline.kernel_us_avg $(python3 -c "import json;print(json.load(open('gpurun_out/bench_prof_frame.json'))['roofline']['kernel_us_avg'])"))"; python3 scripts/ktrace_summary.py gpurun_out/prof_frame 20 1; } > gpurun_out/ktrace_summary.txt
cat gpurun_out/ktrace_summary.txt
rm -rf gpurun_out/prof_encb
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_encb -o run -- python3 scripts/enc_batch_profile.py 64 8 > gpurun_out/enc_batch.log 2>&1 || { tail gpurun_out/enc_batch.log; exit 1; }
cat gpurun_out/enc_batch.log | grep batch
python3 - <<'PY'
import csv
for r in sorted(csv.DictReader(open("gpurun_out/prof_encb/run_kernel_stats.csv")), key=lambda r: -float(r["TotalDurationNs"]))[:6]:
    print(f"{float(r['AverageNs']) / 1e3:9.2f} us  x{r['Calls']:>4}  {r['Name'][:90]}")
PY
python3 -c "import numpy as np, sys; sys.path.insert(0,'.'); from metalhuffman_amd import frames as F; open('gpurun_out/bb.gray','wb').write(np.ascontiguousarray(F.bigbridge()).tobytes())"
timeout -k 10 120 ./host/mh_decode_multi 1 64 20 2048 1536 gpurun_out/bb.gray > gpurun_out/multi.log 2>&1 || { cat gpurun_out/multi.log; exit 1; }
cat gpurun_out/multi.log
rm -f gpurun_out/bb.gray

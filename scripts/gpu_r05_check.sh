# Round-5 final GPU check at HEAD (fail-fast): the library rebuilt and linked on the box from
# this snapshot (build --force), the whole GPU suite on it, smoke, the driver's bench command,
# rocprofv3 kernel traces of each workload's bench command, the encoders' traces, the plain-C
# multi-GPU host.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
sha256sum metalhuffman_amd/libmetalhuffman_amd.so > gpurun_out/build_on_box.log
timeout -k 10 900 python -m metalhuffman_amd.build --force >> gpurun_out/build_on_box.log 2>&1 || { tail -20 gpurun_out/build_on_box.log; exit 1; }
sha256sum metalhuffman_amd/libmetalhuffman_amd.so >> gpurun_out/build_on_box.log
grep -c -- "--offload-arch=gfx950" gpurun_out/build_on_box.log; tail -1 gpurun_out/build_on_box.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log; grep -c PASSED gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
: > gpurun_out/ktrace_summary.txt
for spec in frame:20:5 batch:256:256 tile8192:512:512 tile8192_random:512:512; do
  IFS=: read wl k w <<< "$spec"
  rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_$wl
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$wl -o run -- python3 bench.py --workload $wl --steps $k --warmup $w --no-extras --no-cpu-baseline > gpurun_out/bench_prof_$wl.json 2> gpurun_out/bench_prof_$wl.err || { tail gpurun_out/bench_prof_$wl.err; exit 1; }
  u=$(python3 -c "import json;print(json.load(open('gpurun_out/bench_prof_$wl.json'))['roofline'].get('kernel_us_steady_unit') or 1)")
  { echo "== bench.py --workload $wl --steps $k --warmup $w (profiled line: roofline.kernel_us_avg $(python3 -c "import json;print(json.load(open('gpurun_out/bench_prof_$wl.json'))['roofline']['kernel_us_avg'])"), steady unit $u)"; python3 scripts/ktrace_summary.py gpurun_out/prof_$wl $k $u; } >> gpurun_out/ktrace_summary.txt
done
cat gpurun_out/ktrace_summary.txt
rm -rf gpurun_out/prof_encb
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_encb -o run -- python3 scripts/enc_batch_profile.py 64 8 > gpurun_out/enc_batch.log 2>&1 || { tail gpurun_out/enc_batch.log; exit 1; }
grep batch gpurun_out/enc_batch.log
rm -rf gpurun_out/prof_encode
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_encode -o run -- python3 scripts/enc_profile.py 64 > gpurun_out/enc_profile.log 2>&1 || { tail gpurun_out/enc_profile.log; exit 1; }
python3 - > gpurun_out/encoder_ktrace.txt <<'PY'
import csv
print([l for l in open("gpurun_out/enc_profile.log") if "async encode" in l][-1].strip())
for d in ("prof_encode", "prof_encb"):
    print("==", d)
    for r in sorted(csv.DictReader(open(f"gpurun_out/{d}/run_kernel_stats.csv")), key=lambda r: -float(r["TotalDurationNs"]))[:6]:
        print(f"{float(r['AverageNs']) / 1e3:9.2f} us  x{r['Calls']:>4}  {r['Name'][:90]}")
PY
cat gpurun_out/encoder_ktrace.txt
python3 -c "import numpy as np, sys; sys.path.insert(0,'.'); from metalhuffman_amd import frames as F; open('gpurun_out/bb.gray','wb').write(np.ascontiguousarray(F.bigbridge()).tobytes())"
timeout -k 10 120 ./host/mh_decode_multi 1 64 20 2048 1536 gpurun_out/bb.gray > gpurun_out/multi.log 2>&1 || { cat gpurun_out/multi.log; exit 1; }
grep -v "^RCCL\|^$" gpurun_out/multi.log | tail -3
rm -f gpurun_out/bb.gray

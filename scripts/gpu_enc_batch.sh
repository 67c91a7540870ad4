# Batched encoder: its GPU tests, then a rocprofv3 kernel trace of 8 calls of 64 frames.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode_batch.py tests/test_gpu_encode.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_enc.log 2>&1 || { tail -30 gpurun_out/pytest_enc.log; exit 1; }
tail -1 gpurun_out/pytest_enc.log
rm -rf gpurun_out/prof_encb
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_encb -o run -- python3 scripts/enc_batch_profile.py 64 8 > gpurun_out/enc_batch.log 2>&1 || { tail gpurun_out/enc_batch.log; exit 1; }
grep batch gpurun_out/enc_batch.log
python3 - <<'PY'
import csv
for r in sorted(csv.DictReader(open("gpurun_out/prof_encb/run_kernel_stats.csv")), key=lambda r: -float(r["TotalDurationNs"]))[:4]:
    print(f"{float(r['AverageNs']) / 1e3:9.2f} us  x{r['Calls']:>4}  {r['Name'][:90]}")
PY

# Encoder check: GPU encoder tests, then the fused (default) and four-kernel paths'
# per-kernel times (rocprofv3) and gated device time per BigBridge frame.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_enc.log 2>&1 || { tail -30 gpurun_out/pytest_enc.log; exit 1; }
tail -1 gpurun_out/pytest_enc.log
: > gpurun_out/enc_quick.txt
for k in 2 4; do
  export MH_ENCODE_KERNELS=$k
  rm -rf gpurun_out/prof_enc_k$k
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_enc_k$k -o run -- python3 scripts/enc_profile.py 64 > gpurun_out/enc_k$k.log 2>&1 || { tail gpurun_out/enc_k$k.log; exit 1; }
  timeout -k 10 120 python3 scripts/enc_profile.py 256 > gpurun_out/enc_plain_k$k.log 2>&1 || { tail gpurun_out/enc_plain_k$k.log; exit 1; }
  { echo "== MH_ENCODE_KERNELS=$k"; grep "encode" gpurun_out/enc_plain_k$k.log; python3 - $k <<'PY'
import csv, sys
k = sys.argv[1]
for r in sorted(csv.DictReader(open(f"gpurun_out/prof_enc_k{k}/run_kernel_stats.csv")), key=lambda r: -float(r["AverageNs"])):
    print(f"   {float(r['AverageNs']) / 1e3:8.2f} us  x{r['Calls']:>4}  {r['Name'][:70]}")
PY
  } >> gpurun_out/enc_quick.txt
done
cat gpurun_out/enc_quick.txt

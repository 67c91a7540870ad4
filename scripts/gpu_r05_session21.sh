# Round 5, GPU session 21: the lazy-refill default under new cases -- the refill-extreme GPU
# tests, then a 5-minute randomized parity sweep at this HEAD (new case ids from 200000).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -v -k "refill_extremes or small_launch or long_codes" --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_refill_extremes.log 2>&1 || { tail -30 gpurun_out/r05_pytest_refill_extremes.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r05_pytest_refill_extremes.log | tail -12
MH_STRESS_SECONDS=300 MH_STRESS_FIRST_CASE=200000 bash scripts/gpu_stress_long.sh
cp gpurun_out/stress_long.log gpurun_out/r05_stress_head2.log
tail -4 gpurun_out/r05_stress_head2.log

# A longer randomized GPU parity sweep (decode + single-frame and batched GPU encode) at HEAD,
# starting past the cases the default test run covers.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
export MH_STRESS_SECONDS=${MH_STRESS_SECONDS:-420} MH_STRESS_FIRST_CASE=${MH_STRESS_FIRST_CASE:-30000}
timeout -k 10 560 python -u -m pytest tests/test_gpu_stress.py -x -q -s --timeout 540 --timeout-method thread > gpurun_out/stress_long.log 2>&1 || { tail -30 gpurun_out/stress_long.log; exit 1; }
grep "stress\] done" gpurun_out/stress_long.log; tail -1 gpurun_out/stress_long.log

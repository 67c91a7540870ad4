# Encoder verification: the GPU encoder tests, then the randomized parity sweep (decode +
# single-frame and batched GPU encode) for MH_STRESS_SECONDS.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode_batch.py tests/test_gpu_encode.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_enc.log 2>&1 || { tail -30 gpurun_out/pytest_enc.log; exit 1; }
tail -1 gpurun_out/pytest_enc.log
export MH_STRESS_SECONDS=${MH_STRESS_SECONDS:-90}
timeout -k 10 400 python -u -m pytest tests/test_gpu_stress.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/stress.log 2>&1 || { tail -30 gpurun_out/stress.log; exit 1; }
grep "stress\] done" gpurun_out/stress.log; tail -1 gpurun_out/stress.log

# Pair-table batch kernel: full GPU parity, then A/B (default = pair kernel) vs variants.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
VARIANTS="default nopair pw10 default nopair pw10" WLS="batch tile8192 tile8192_random" STEPS=200 timeout -k 10 900 bash scripts/gpu_ab.sh

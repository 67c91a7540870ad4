# Round 5, GPU session 1: the whole GPU suite on this tree (split batch loop, lane pairs
# in the diagnostic library, fork-safe CPU pool, encoder tile tails, rank devices), then
# the batch-kernel bisect (scripts/gpu_r05_bisect.sh, no PMC).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r05_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r05_pytest_gpu.log
bash scripts/gpu_r05_bisect.sh

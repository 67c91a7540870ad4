# Full GPU parity, then an interleaved A/B of the default build against the variants in
# ab on the batch, 8192^2 and random workloads.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
V=$(ls ab | sed 's/^lib_//; s/\.so$//' | tr '\n' ' ')
VARIANTS="default $V default $V" WLS="${WLS:-batch tile8192 tile8192_random}" STEPS=200 timeout -k 10 900 bash scripts/gpu_ab.sh

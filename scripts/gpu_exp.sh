# Experiment round: parity on the default library, A/B of variants, diag timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -20; exit 1; }
STEPS=${STEPS:-400} bash scripts/gpu_ab.sh || exit 1
if [ -f metalhuffman_amd/_variants/lib_diag.so ]; then
  export MH_LIB=$GRAFT_REPO_ROOT/metalhuffman_amd/_variants/lib_diag.so
  timeout -k 10 300 python scripts/diag_stamps.py --batch 1 > gpurun_out/diag1.txt 2>&1 || exit 1
  timeout -k 10 300 python scripts/diag_stamps.py --batch 64 > gpurun_out/diag64.txt 2>&1 || exit 1
  cat gpurun_out/diag1.txt gpurun_out/diag64.txt
fi

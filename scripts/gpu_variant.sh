# Parity of a variant library, then A/B against the default and a diag timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=${V:?set V=<variant name>}
MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$V.so timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_$V.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu_$V.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gpu_$V.log | head -20; exit 1; }
VARIANTS="${VARIANTS:-default $V default $V}" WLS="${WLS:-batch tile8192 tile8192_random}" STEPS=${STEPS:-200} bash scripts/gpu_ab.sh || exit 1
if [ -n "${DIAG:-}" ]; then
  MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$DIAG.so timeout -k 10 120 python scripts/diag_stamps.py --batch 64 --tag _$DIAG > gpurun_out/diag64_$DIAG.txt 2>&1 || exit 1
  cat gpurun_out/diag64_$DIAG.txt
fi

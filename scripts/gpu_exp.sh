# Experiment round: parity on the default library, A/B of variants, diag timelines.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -20; exit 1; }
STEPS=${STEPS:-400} bash scripts/gpu_ab.sh || exit 1
for d in ${DIAGS:-diag}; do
  [ -f ab/lib_$d.so ] || continue
  export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$d.so
  timeout -k 10 300 python scripts/diag_stamps.py --batch 64 ${DIAG_ARGS:-} --tag _$d > gpurun_out/diag64_$d.txt 2>&1 || exit 1
  echo "== $d"; tail -7 gpurun_out/diag64_$d.txt
done
if [ -n "${PROF_FRAME:-}" ]; then
  unset MH_LIB
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ktrace -o kt -- python3 bench.py --workload frame --steps 200 --warmup 20 --no-extras --no-cpu-baseline > gpurun_out/ktrace.log 2>&1 || exit 1
fi

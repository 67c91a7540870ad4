# Config-3 grid balance A/B: workgroup width / resident
# workgroups per CU for the persistent batch kernel, timed by bench.py, plus the
# per-wave phase stamps of the diagnostic builds (loop end per wave) on tile8192.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
VARIANTS="default w8g2 w4 w7 w6" WLS="tile8192 tile8192_random batch" STEPS=256 \
  timeout -k 10 900 bash scripts/gpu_ab.sh > gpurun_out/grid_ab.txt 2>&1 || { cat gpurun_out/grid_ab.txt; exit 1; }
cat gpurun_out/grid_ab.txt
for v in w8 w8g2 w4; do
  echo "== stamps $v (tile8192)"
  MH_LIB=$GRAFT_REPO_ROOT/ab/lib_diag_$v.so timeout -k 10 120 python scripts/diag_stamps.py --tile8192 --tag _$v || exit 1
done

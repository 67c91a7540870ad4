# Round 5, GPU session 23: flat 8-bit path variants on the uniform-random 8192^2 tile --
# default (per-lane loads, one tile of codes ahead), f8staged (batch_loop's coalesced span
# loads and LDS stage, byte arithmetic from the stage), f8prio (default + wave priority by
# tiles left), noflat8 (the general flat step); flat tests through f8staged first.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_flat8_variants_ab.txt
: > $OUT
MH_LIB=$GRAFT_REPO_ROOT/ab/lib_f8staged.so timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -q -k "flat" --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_f8staged.log 2>&1
rc=$?
tail -2 gpurun_out/r05_pytest_f8staged.log >> $OUT
[ $rc -le 1 ] || exit 1
STAGED_OK=$rc
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'])"; }
for rep in 1 2 3; do
  for v in default f8staged f8prio noflat8; do
    [ "$v" = f8staged ] && [ "$STAGED_OK" != 0 ] && continue
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload tile8192_random --steps 64 --warmup 32 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_flat8_variants_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v tile8192_random $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
cat $OUT

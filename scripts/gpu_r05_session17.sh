# Round 5, GPU session 17: why the single-frame decode chain runs ~0.45 us longer cold than warm.
# Stamps with core-clock cycles (MH_DIAG_CLOCK), the same with every row store dropped, and with
# an entry-time touch of the tile's output rows and codes page (MH_SMALL_TOUCH); then the driver's
# frame command, default vs touch vs lazy refill (MH_SMALL_LAZY), interleaved x 3, after the
# lazy variant's decode parity tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_chain_cold_ab.txt
: > $OUT
echo "== pytest decode, lazy refill" >> $OUT
MH_LIB=$GRAFT_REPO_ROOT/ab/lib_lazy.so timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_stress.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_lazy.log 2>&1
rc=$?
tail -3 gpurun_out/r05_pytest_lazy.log >> $OUT
echo "pytest rc $rc" >> $OUT
# a wrong-output failure (1) is a result; a fault, abort or time limit ends the call
[ $rc -le 1 ] || exit 1
LAZY_OK=$rc
for v in stampclk stampclk_nostore stampclk_touch stampclk_lazy; do
  export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so
  { echo "== $v --cold"; timeout -k 10 180 python3 scripts/diag_stamps.py --cold --clock --tag _$v 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
  { echo "== $v warm"; timeout -k 10 180 python3 scripts/diag_stamps.py --clock --tag _$v 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
  echo "$v stamps done"
done
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'warm', d.get('warm_value'))"; }
for rep in 1 2 3; do
  for v in default touch lazy; do
    [ "$v" = lazy ] && [ "$LAZY_OK" != 0 ] && continue
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_chain_cold_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
cat $OUT

# Round 5, GPU session 29: the lazy step's next-word read as a broadcast for lanes that did not
# refill (MH_SMALL_LAZY_BCAST=1, ab/lib_lzbc.so: only refilling lanes' reads can conflict; the
# read's select deferred one step). Decode tests through it, then the driver's frame command,
# default vs lzbc, interleaved x 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_lazy_bcast_ab.txt
: > $OUT
MH_LIB=$GRAFT_REPO_ROOT/ab/lib_lzbc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_stress.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_lzbc.log 2>&1
rc=$?
tail -2 gpurun_out/r05_pytest_lzbc.log >> $OUT
[ $rc -le 1 ] || exit 1
[ $rc -eq 0 ] || { cat $OUT; exit 0; }
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'])"; }
for rep in 1 2 3 4; do
  for v in default lzbc; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_lazy_bcast_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
cat $OUT

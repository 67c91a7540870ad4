# Round 5, GPU session 30: the lazy step reading the next code word at even steps only
# (MH_SMALL_LAZY_HALF=1, ab/lib_lzhalf.so: half the stage reads; wa changes only at a refill and
# no refill follows a refill). Decode tests through it, then the driver's frame command, default
# vs lzhalf, interleaved x 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_lazy_half_ab.txt
: > $OUT
MH_LIB=$GRAFT_REPO_ROOT/ab/lib_lzhalf.so timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_stress.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_lzhalf.log 2>&1
rc=$?
tail -2 gpurun_out/r05_pytest_lzhalf.log >> $OUT
[ $rc -le 1 ] || exit 1
[ $rc -eq 0 ] || { cat $OUT; exit 0; }
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'])"; }
for rep in 1 2 3 4; do
  for v in default lzhalf; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_lazy_half_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
cat $OUT

# Round 5, GPU session 16: the single-frame kernel with its eight row stores issued after the
# whole block (8 x 2 registers held) instead of after each row, so no store issues between
# the steps of the chain (cold, the chain ran 3.16 us vs 2.68 us warm); decode tests with
# the variant, then the driver's frame command interleaved x 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
MH_LIB=$GRAFT_REPO_ROOT/ab/lib_defer.so timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05_pytest_defer.log 2>&1 || { tail -40 gpurun_out/r05_pytest_defer.log; exit 1; }
tail -1 gpurun_out/r05_pytest_defer.log
OUT=gpurun_out/r05_defer_ab.txt
: > $OUT
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'warm', d.get('warm_value'))"; }
for rep in 1 2 3 4; do
  for v in default defer; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_defer_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
done
cat $OUT

# Round 5, GPU session 15: the single-frame kernel with its 8-row loop rolled (1,203 instead
# of 4,751 instructions: every launch refetches its code after the dispatch's cache
# invalidation) vs the unrolled default; decode tests with the variant, then the driver's
# frame command interleaved x 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
MH_LIB=$GRAFT_REPO_ROOT/ab/lib_rolled.so timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05_pytest_rolled.log 2>&1 || { tail -40 gpurun_out/r05_pytest_rolled.log; exit 1; }
tail -1 gpurun_out/r05_pytest_rolled.log
OUT=gpurun_out/r05_rolled_ab.txt
: > $OUT
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'warm', d.get('warm_value'))"; }
for rep in 1 2 3 4; do
  for v in default rolled; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_rolled_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
done
cat $OUT

# Round 5, GPU session 18: the lazy-refill step (MH_SMALL_LAZY=1, ab/lib_lazy.so) -- every GPU
# test through it, then the driver's frame command default vs lazy, interleaved x 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_lazy_ab.txt
: > $OUT
echo "== pytest -m gpu, lazy refill library" >> $OUT
MH_LIB=$GRAFT_REPO_ROOT/ab/lib_lazy.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_lazy.log 2>&1 || { tail -5 gpurun_out/r05_pytest_lazy.log >> $OUT; exit 1; }
tail -2 gpurun_out/r05_pytest_lazy.log >> $OUT
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'warm', d.get('warm_value'))"; }
for rep in 1 2 3 4; do
  for v in default lazy; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_lazy_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
cat $OUT

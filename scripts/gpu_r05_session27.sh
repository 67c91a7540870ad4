# Round 5, GPU session 27: the flat 8-bit batch path on the uniform-random 8192^2 tile (16,384
# tiles, 2.67 per wave): default (one tile of codes ahead), f8aux18 (write-through row stores),
# f8g2 (two tiles per round trip, flat8_loop_grouped), f8g2aux18; the flat tests through f8g2
# first; interleaved x 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_flat8_group_ab.txt
: > $OUT
MH_LIB=$GRAFT_REPO_ROOT/ab/lib_f8g2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -q -k "flat" --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_f8g2.log 2>&1
rc=$?
tail -2 gpurun_out/r05_pytest_f8g2.log >> $OUT
[ $rc -le 1 ] || exit 1
G_OK=$rc
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'])"; }
for rep in 1 2 3; do
  for v in default f8aux18 f8g2 f8g2aux18; do
    case $v in f8g2*) [ "$G_OK" != 0 ] && continue;; esac
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload tile8192_random --steps 64 --warmup 32 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_flat8_group_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v tile8192_random $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
cat $OUT

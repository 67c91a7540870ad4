# Round 5, GPU session 24: flat 8-bit tables in the single-frame kernel too (byte arithmetic
# from the staged span). The whole GPU suite, then one-frame launches of uniform-random
# 2048x1536 frames (time_frame.py --random, graph of 200 launches) and the driver's config-2
# frame command as a control, default vs noflat8 (MH_FLAT8=0), interleaved x 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_flat8_small_ab.txt
: > $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05_pytest_flat8_all.log 2>&1 || { tail -30 gpurun_out/r05_pytest_flat8_all.log; exit 1; }
tail -1 gpurun_out/r05_pytest_flat8_all.log >> $OUT
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'])"; }
for rep in 1 2 3; do
  for v in default noflat8; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    timeout -k 10 120 python3 scripts/time_frame.py --random --tag $v 2>>gpurun_out/r05_flat8_small_ab.err | tail -1 >> $OUT || { echo "$v FAILED" >> $OUT; exit 1; }
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_flat8_small_ab.err) || { echo "$v frame FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
cat $OUT

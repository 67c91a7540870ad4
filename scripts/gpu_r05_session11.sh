# Round 5, GPU session 11: kernarg preload for the decode kernels (the leading scalar
# arguments in SGPRs at wave launch): decode GPU tests, then default vs decprev (the
# kernels taking only the DecodeArgs struct: nothing preloaded), interleaved: the driver's
# frame command (20 steps) x 4, batch and 8192^2 x 2.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_lane_pairs.py tests/test_check.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05_pytest_dec.log 2>&1 || { tail -40 gpurun_out/r05_pytest_dec.log; exit 1; }
tail -1 gpurun_out/r05_pytest_dec.log
OUT=gpurun_out/r05_preload_ab.txt
: > $OUT
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'warm', d.get('warm_value'), 'ungated', d.get('ungated_value'))"; }
for rep in 1 2 3 4; do
  for v in default decprev; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    specs="frame:20:5"
    if [ $rep -le 2 ]; then specs="frame:20:5 batch:64:16 tile8192:64:16"; fi
    for spec in $specs; do
      IFS=: read wl k w <<< "$spec"
      r=$(timeout -k 10 150 python bench.py --workload $wl --steps $k --warmup $w --no-extras --no-cpu-baseline 2>>gpurun_out/r05_preload_ab.err) || { echo "$v $wl FAILED" >> $OUT; exit 1; }
      echo "$v $wl $(echo "$r" | line)" >> $OUT
    done
  done
  echo "rep $rep done"
done
unset MH_LIB
cat $OUT

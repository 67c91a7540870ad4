# Round 5, GPU session 22: the batch kernel's flat 8-bit path (byte arithmetic, no table
# lookups; MH_BATCH_FLAT8). The decode GPU tests (new flat8 formats included), then the
# uniform-random 8192^2 tile (config 3 stress) and the batch / 8192^2 BigBridge tile as a
# control, default vs noflat8 (the general flat step), interleaved x 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_flat8_ab.txt
: > $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_check.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_flat8.log 2>&1
rc=$?
tail -3 gpurun_out/r05_pytest_flat8.log >> $OUT
echo "pytest rc $rc" >> $OUT
[ $rc -eq 0 ] || { tail -40 gpurun_out/r05_pytest_flat8.log; exit 1; }
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'])"; }
for rep in 1 2 3; do
  for wl in tile8192_random batch; do
    for v in default noflat8; do
      if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
      r=$(timeout -k 10 150 python bench.py --workload $wl --steps 64 --warmup 32 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_flat8_ab.err) || { echo "$v $wl FAILED" >> $OUT; exit 1; }
      echo "$v $wl $(echo "$r" | line)" >> $OUT
    done
  done
  echo "rep $rep done"
done
cat $OUT

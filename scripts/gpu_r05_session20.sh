# Round 5, GPU session 20: the batch kernel with the single-level 14-bit table for tables whose
# longest code is 14 bits (MH_BATCH_L14=1, ab/lib_bl14.so: no escape test, 2 workgroups per CU
# by LDS instead of 3). Decode GPU tests through it, then batch / tile8192 / tile8192_random,
# default vs bl14, interleaved x 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_batch_l14_ab.txt
: > $OUT
echo "== pytest decode + stress, bl14 library" >> $OUT
MH_LIB=$GRAFT_REPO_ROOT/ab/lib_bl14.so timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_stress.py tests/test_check.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_bl14.log 2>&1
rc=$?
tail -3 gpurun_out/r05_pytest_bl14.log >> $OUT
[ $rc -le 1 ] || exit 1
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'])"; }
for rep in 1 2 3; do
  for wl in batch tile8192 tile8192_random; do
    for v in default bl14; do
      if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
      r=$(timeout -k 10 150 python bench.py --workload $wl --steps 64 --warmup 32 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_batch_l14_ab.err) || { echo "$v $wl FAILED" >> $OUT; exit 1; }
      echo "$v $wl $(echo "$r" | line)" >> $OUT
    done
  done
  echo "rep $rep done"
done
cat $OUT

# Round 4 A/B 4: the single-frame kernel's table barrier as an LDS-only barrier (default) vs
# __syncthreads (head: its fence waits for the span loads too). bench.py --workload frame
# (cold regions), interleaved three times, then the decode GPU tests on the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r04_ab4.txt
: > $OUT
for rep in 1 2 3; do
  for v in default head; do
    if [ $v = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    for spec in frame:20:5 frame:200:20; do
      IFS=: read wl k w <<< "$spec"
      r=$(timeout -k 10 300 python bench.py --workload $wl --steps $k --warmup $w --no-extras --no-cpu-baseline 2>>gpurun_out/r04_ab4.err) || { echo "$v $wl FAILED" >> $OUT; exit 1; }
      echo "$v $wl:$k $r" | python3 -c "import sys,json; l=sys.stdin.read().split(' ',2); d=json.loads(l[2]); print(l[0], l[1], 'value', d['value'], 'warm', d.get('warm_value'), 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'])" >> $OUT
    done
  done
done
unset MH_LIB
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_dec.log 2>&1 || { tail -30 gpurun_out/pytest_dec.log; exit 1; }
tail -1 gpurun_out/pytest_dec.log >> $OUT
cat $OUT

# Round 4 A/B 3: batch prologue with the table loaded first and an LDS-only barrier (default)
# vs the round's head; stamps of the cold 8192^2 tile; the batched encoder's tests and trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_enc_batch.sh || exit 1
OUT=gpurun_out/r04_ab3.txt
: > $OUT
for rep in 1 2; do
  for v in default head; do
    if [ $v = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    for spec in batch:64:16 tile8192:64:16 tile8192_random:64:16; do
      IFS=: read wl k w <<< "$spec"
      r=$(timeout -k 10 300 python bench.py --workload $wl --steps $k --warmup $w --no-extras --no-cpu-baseline 2>>gpurun_out/r04_ab3.err) || { echo "$v $wl FAILED" >> $OUT; exit 1; }
      echo "$v $wl $r" | python3 -c "import sys,json; l=sys.stdin.read().split(' ',2); d=json.loads(l[2]); print(l[0], l[1], 'value', d['value'], 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'])" >> $OUT
    done
  done
done
export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_stamps2.so
{ echo "== stamps --tile8192 --cold (table first, LDS-only barrier)"; timeout -k 10 180 python3 scripts/diag_stamps.py --tile8192 --cold 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
unset MH_LIB
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_dec.log 2>&1 || { tail -30 gpurun_out/pytest_dec.log; exit 1; }
tail -1 gpurun_out/pytest_dec.log >> $OUT
cat $OUT

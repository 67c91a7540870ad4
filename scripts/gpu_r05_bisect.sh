# Round 5: bisect of the round-4 batch-kernel regression on ONE box,
# interleaved: r03 head (f433465), 8397e6d (single flavour-switched loop + kernel args),
# HEAD r04 (7dc48b7 prologue), and "split" (the r05 tree: r04 prologue + one loop
# instantiation per flavour); workloads batch / tile8192 / tile8192_random; then one
# PMC pass per variant on the batch.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_bisect.txt
: > $OUT
VARS=${VARS:-"r03 c8397 head split"}
for rep in 1 2; do
  for v in $VARS; do
    if [ $v = split ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    for wl in ${WLS:-batch tile8192 tile8192_random}; do
      r=$(timeout -k 10 150 python bench.py --workload $wl --steps 64 --warmup 16 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_bisect.err) || { echo "$v $wl FAILED" >> $OUT; exit 1; }
      echo "$v $wl $r" | python3 -c "import sys,json; l=sys.stdin.read().split(' ',2); d=json.loads(l[2]); print(l[0], l[1], 'value', d['value'], 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'])" >> $OUT
      echo "rep $rep $v $wl done"
    done
  done
done
if [ -n "$PMC" ]; then
for v in $VARS; do
  if [ $v = split ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
  rm -rf gpurun_out/pmc_$v; mkdir -p gpurun_out/pmc_$v
  timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_$v/pmc1 -o run -- python3 bench.py --workload batch --steps 16 --warmup 2 --no-extras --no-cpu-baseline > gpurun_out/pmc_$v.log 2>&1 || { tail gpurun_out/pmc_$v.log; exit 1; }
  { echo "== PMC $v batch (mh_decode_kernel, per dispatch)"; python3 scripts/pmc_summary.py gpurun_out/pmc_$v mh_decode_kernel 2; } >> $OUT
  echo "pmc $v done"
done
fi
cat $OUT

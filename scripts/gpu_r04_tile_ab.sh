# Round 4: (1) VMEM-refill A/B on the batch kernel: bench + one PMC pass
# each; (2) per-wave phase stamps of the 8192^2 tile and the 64-frame batch, cold and warm
# (start / steady / drain).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r04_ab.txt
: > $OUT
for rep in 1 2; do
  for v in default vmemrefill; do
    if [ $v = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    for wl in batch tile8192; do
      r=$(timeout -k 10 300 python bench.py --workload $wl --steps 64 --warmup 16 --no-extras --no-cpu-baseline 2>>gpurun_out/r04_ab.err) || { echo "$v $wl FAILED" >> $OUT; exit 1; }
      echo "$v $wl $r" | python3 -c "import sys,json; l=sys.stdin.read().split(' ',2); d=json.loads(l[2]); print(l[0], l[1], 'value', d['value'], 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'])" >> $OUT
    done
  done
done
for v in default vmemrefill; do
  if [ $v = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
  rm -rf gpurun_out/pmc_$v; mkdir -p gpurun_out/pmc_$v
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_$v/pmc1 -o run -- python3 bench.py --workload batch --steps 16 --warmup 2 --no-extras --no-cpu-baseline > gpurun_out/pmc_$v.log 2>&1 || { tail gpurun_out/pmc_$v.log; exit 1; }
  { echo "== PMC $v batch (mh_decode_kernel, per dispatch)"; python3 scripts/pmc_summary.py gpurun_out/pmc_$v mh_decode_kernel 2; } >> $OUT
done
unset MH_LIB
export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_stamps.so
for args in "--tile8192 --cold" "--tile8192" "--batch 64 --cold"; do
  { echo "== stamps $args"; timeout -k 10 180 python3 scripts/diag_stamps.py $args 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
done
cat $OUT

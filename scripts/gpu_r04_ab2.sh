# Round 4 A/B: the batch prologue's fixed table loads (default) vs the previous head; stamps
# of the new prologue on the cold 8192^2 tile; PMC of the batched encoder's kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r04_ab2.txt
: > $OUT
for rep in 1 2; do
  for v in default head; do
    if [ $v = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    for spec in batch:64:16 tile8192:64:16 tile8192_random:64:16 frame:20:5; do
      IFS=: read wl k w <<< "$spec"
      r=$(timeout -k 10 300 python bench.py --workload $wl --steps $k --warmup $w --no-extras --no-cpu-baseline 2>>gpurun_out/r04_ab2.err) || { echo "$v $wl FAILED" >> $OUT; exit 1; }
      echo "$v $wl $r" | python3 -c "import sys,json; l=sys.stdin.read().split(' ',2); d=json.loads(l[2]); print(l[0], l[1], 'value', d['value'], 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'])" >> $OUT
    done
  done
done
export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_stamps2.so
{ echo "== stamps --tile8192 --cold (fixed table loads)"; timeout -k 10 180 python3 scripts/diag_stamps.py --tile8192 --cold 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
unset MH_LIB
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"; do
  i=$((i+1)); rm -rf gpurun_out/pmc_enc/pmc$i
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_enc/pmc$i -o run -- python3 scripts/enc_batch_profile.py 64 2 > gpurun_out/pmc_enc$i.log 2>&1 || { tail gpurun_out/pmc_enc$i.log; exit 1; }
done
for k in enc_split_kernel enc_tree_batch_kernel enc_pack_batch_kernel; do
  { echo "== PMC $k (per dispatch)"; python3 scripts/pmc_summary.py gpurun_out/pmc_enc $k 1; } >> $OUT
done
cat $OUT

# LDS / VALU counters of the batch workload, pair kernel (default) vs single-step (nopair variant).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
B="python3 bench.py --workload batch --steps 10 --warmup 2 --no-extras --no-cpu-baseline"
for v in default nopair; do
  if [ $v = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
  rm -rf $OUT/pmcab_$v
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmcab_$v/pmc1 -o run -- $B > $OUT/pmcab_$v.log 2>&1 || { echo "pmc $v failed"; tail $OUT/pmcab_$v.log; exit 1; }
  echo "== $v"
  python3 scripts/pmc_summary.py $OUT/pmcab_$v decode_ 2
done

# One LDS/VALU counter pass per build (default + $V) over a workload: does an A/B
# change the counters the way its model says? -> gpurun_out/pmc_ab.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:?set V=<variant>}
WL=${WL:-batch}
: > gpurun_out/pmc_ab.txt
for v in default $V; do
  if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
  for grp in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES"; do
    rm -rf gpurun_out/pmcab_$v
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmcab_$v -o run -- python3 bench.py --workload $WL --steps 10 --warmup 2 --no-extras --no-cpu-baseline > gpurun_out/pmcab_$v.log 2>&1 || { echo "pmc $v failed"; tail gpurun_out/pmcab_$v.log; exit 1; }
    { echo "== $v $WL"; python3 scripts/pmc_summary.py gpurun_out/pmcab_$v mh_decode_kernel 2; } >> gpurun_out/pmc_ab.txt
  done
done
cat gpurun_out/pmc_ab.txt

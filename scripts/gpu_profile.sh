# PMC counter passes over the batch workload (one pass per counter group).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${OUT:-$GRAFT_REPO_ROOT/gpurun_out}
mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
B="python3 bench.py --workload ${WL:-batch} --steps 10 --warmup 2 --no-extras --no-cpu-baseline"
i=0
# PMC_GROUPS="grp1;grp2" (space-separated counters per group) replaces the default groups
DEFAULT_GROUPS=$(cat <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
GROUPS
)
if [ -n "$PMC_GROUPS" ]; then ALL_GROUPS=$(echo "$PMC_GROUPS" | tr ';' '\n'); else ALL_GROUPS=$DEFAULT_GROUPS; fi
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- $B > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done <<< "$ALL_GROUPS"
echo "profile done ($i passes)"

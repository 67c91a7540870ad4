# Round 5, GPU session 31: per-wave stamps with core-clock cycles of the final single-frame
# kernel (lazy refill, even-step next-word reads): bench-style cold shuffled frames and the warm
# natural frame.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_final_stamps.txt
: > $OUT
export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_stampclk.so
{ echo "== final --cold"; timeout -k 10 180 python3 scripts/diag_stamps.py --cold --clock --tag _final 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
{ echo "== final warm (natural frame)"; timeout -k 10 180 python3 scripts/diag_stamps.py --clock --tag _final 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
cat $OUT

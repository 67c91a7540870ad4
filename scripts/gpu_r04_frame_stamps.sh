# Cold and warm phase stamps of the single-frame launch (config 2) from a MH_DIAG_STAMPS=1 build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_stamps.so
OUT=gpurun_out/r04_frame_stamps.txt
{ echo "== stamps single frame --cold"; timeout -k 10 180 python3 scripts/diag_stamps.py --cold 2>&1 | grep -v amdgpu.ids; } > $OUT || exit 1
{ echo "== stamps single frame (warm)"; timeout -k 10 180 python3 scripts/diag_stamps.py 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
cat $OUT

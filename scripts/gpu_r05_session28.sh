# Round 5, GPU session 28: an 8-minute randomized parity sweep at the final HEAD, new case ids
# from 400000.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
MH_STRESS_SECONDS=480 MH_STRESS_FIRST_CASE=400000 bash scripts/gpu_stress_long.sh
cp gpurun_out/stress_long.log gpurun_out/r05_stress_head4.log
tail -4 gpurun_out/r05_stress_head4.log

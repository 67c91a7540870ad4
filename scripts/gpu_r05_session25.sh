# Round 5, GPU session 25: a 5-minute randomized parity sweep at the final HEAD (the flat 8-bit
# paths included: the sweep's "uniform" frames), new case ids from 300000.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
MH_STRESS_SECONDS=300 MH_STRESS_FIRST_CASE=300000 bash scripts/gpu_stress_long.sh
cp gpurun_out/stress_long.log gpurun_out/r05_stress_head3.log
tail -4 gpurun_out/r05_stress_head3.log

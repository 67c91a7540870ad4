# Round 5, GPU session 5: H2D probe (config 5: is one copy stream the limit?), the 2-rank
# gloo rehearsal of the N > 1 bench path (rank_devices at world 2), and a randomized parity
# sweep at this HEAD (decode paths + single-frame and batched GPU encode).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python3 scripts/h2d_probe.py > gpurun_out/r05_h2d_probe.txt 2>&1 || { cat gpurun_out/r05_h2d_probe.txt; exit 1; }
cat gpurun_out/r05_h2d_probe.txt
bash scripts/gpu_rehearse_n2.sh > gpurun_out/r05_rehearse_n2.txt 2>&1 || { cat gpurun_out/r05_rehearse_n2.txt; exit 1; }
cat gpurun_out/r05_rehearse_n2.txt
MH_STRESS_SECONDS=300 MH_STRESS_FIRST_CASE=120000 bash scripts/gpu_stress_long.sh
cp gpurun_out/stress_long.log gpurun_out/r05_stress.log

set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_check.sh > gpurun_out/check.out 2>&1 || { tail -30 gpurun_out/check.out; exit 1; }
tail -5 gpurun_out/check.out
bash scripts/gpu_bench20.sh > gpurun_out/b20.out 2>&1 || { tail -30 gpurun_out/b20.out; exit 1; }
cat gpurun_out/b20_rep.txt

# SQ / LDS / TCC counter passes (scripts/gpu_profile.sh's groups) over the three decode
# workloads -> gpurun_out/pmc_<wl>/ and a per-workload summary in gpurun_out/pmc_kernels.txt.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/pmc_kernels.txt
for spec in batch:mh_decode_kernel frame:mh_decode_small_kernel tile8192:mh_decode_kernel; do
  IFS=: read wl kern <<< "$spec"
  rm -rf gpurun_out/pmc_$wl
  WL=$wl OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$wl bash scripts/gpu_profile.sh || exit 1
  { echo "== $wl ($kern)"; python3 scripts/pmc_summary.py gpurun_out/pmc_$wl $kern 2; } >> gpurun_out/pmc_kernels.txt
done
cat gpurun_out/pmc_kernels.txt

# Encoder paths A/B (one-launch vs two-launch) on BigBridge-shuffled frames: time per
# frame (scripts/enc_profile.py) and PMC traffic (FETCH_SIZE x2 + WRITE_SIZE, one
# --pmc pass per counter) -> gpurun_out/enc_paths.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/enc_paths
rm -rf $OUT; mkdir -p $OUT
: > gpurun_out/enc_paths.txt
for p in 2 1 2 1; do
  echo "== MH_ENCODE_KERNELS=$p" >> gpurun_out/enc_paths.txt
  MH_ENCODE_KERNELS=$p timeout -k 10 120 python3 scripts/enc_profile.py 32 2>&1 | grep -v amdgpu.ids >> gpurun_out/enc_paths.txt || exit 1
done
for p in 2 1; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    MH_ENCODE_KERNELS=$p timeout -k 10 120 rocprofv3 --pmc $ctr --output-format csv -d $OUT/p${p}/encode_$ctr -o run -- \
      python3 scripts/enc_profile.py 16 > $OUT/p${p}_$ctr.log 2>&1 || { echo "pmc $p $ctr failed"; tail -5 $OUT/p${p}_$ctr.log; exit 1; }
  done
  echo "== PMC, MH_ENCODE_KERNELS=$p" >> gpurun_out/enc_paths.txt
  python3 scripts/traffic_summary.py $OUT/p${p} >> gpurun_out/enc_paths.txt || exit 1
done
cat gpurun_out/enc_paths.txt

# HBM traffic per decode launch from PMC counters (separate --pmc passes per counter),
# for each bench workload -> gpurun_out/traffic.json (copy into profiles/ to commit).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/traffic
rm -rf $OUT; mkdir -p $OUT
for wl in ${WLS-frame batch tile8192 tile8192_random}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d $OUT/${wl}_$ctr -o run -- \
      python3 bench.py --workload $wl --steps 20 --warmup 2 --no-extras --no-cpu-baseline --no-graph \
      > $OUT/${wl}_$ctr.log 2>&1 || { echo "pmc $wl $ctr failed"; tail -5 $OUT/${wl}_$ctr.log; exit 1; }
  done
done
# the GPU encoder's two kernels (split, code) on BigBridge-shuffled frames
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d $OUT/encode_$ctr -o run -- \
    python3 scripts/enc_profile.py 16 > $OUT/encode_$ctr.log 2>&1 || { echo "pmc encode $ctr failed"; tail -5 $OUT/encode_$ctr.log; exit 1; }
done
python3 scripts/traffic_summary.py $OUT > gpurun_out/traffic.json && cat gpurun_out/traffic.json

# Round 5, GPU session 6: does the cold-region flush itself slow the first launch of a
# region? bench.py's flush is a 512 MiB device copy (dirty lines left behind); A/B against
# a read-only eviction (MH_BENCH_FLUSH=read: a reduction over 1 GiB, nothing dirty), on
# the driver's frame command and the batch / tile workloads, interleaved; then per-wave
# stamps of the first launch after each kind of flush.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_flush_ab.txt
: > $OUT
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'warm', d.get('warm_value'))"; }
for rep in 1 2 3; do
  for mode in copy read; do
    for spec in frame:20:5 batch:64:16 tile8192:64:16; do
      IFS=: read wl k w <<< "$spec"
      r=$(MH_BENCH_FLUSH=$mode timeout -k 10 150 python bench.py --workload $wl --steps $k --warmup $w --no-extras --no-cpu-baseline 2>>gpurun_out/r05_flush_ab.err) || { echo "$mode $wl FAILED" >> $OUT; exit 1; }
      echo "$mode $wl $(echo "$r" | line)" >> $OUT
    done
  done
  echo "rep $rep done"
done
export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_stamps.so
for mode in copy read; do
  { echo "== stamps single frame --cold, flush $mode"; MH_BENCH_FLUSH=$mode timeout -k 10 180 python3 scripts/diag_stamps.py --cold 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
done
cat $OUT

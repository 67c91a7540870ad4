# Round 5, GPU session 19: lazy refill now the default. A codes-page touch at entry
# (MH_SMALL_TOUCH=2: one load per wave at the tile's linear share of the codes, in flight with
# the block offsets) -- stamps cold, then the driver's frame command default vs touch2 vs the
# old eager refill (nolazy), interleaved x 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_touch2_ab.txt
: > $OUT
for v in stampclk stampclk_touch2; do
  export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so
  { echo "== $v --cold"; timeout -k 10 180 python3 scripts/diag_stamps.py --cold --clock --tag _$v 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
  echo "$v stamps done"
done
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'warm', d.get('warm_value'))"; }
for rep in 1 2 3; do
  for v in default touch2 nolazy; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_touch2_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
cat $OUT

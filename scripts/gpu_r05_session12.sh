# Round 5, GPU session 12: the single-frame kernel's workgroup width again after the kernarg
# preload (4 waves = one per SIMD, default; 8 = two per SIMD, half the workgroups; 2), on the
# driver's frame command, interleaved x 3; then per-wave stamps of the current kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_small_wg_ab.txt
: > $OUT
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'warm', d.get('warm_value'))"; }
for rep in 1 2 3; do
  for v in default small8 small2; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_small_wg_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_stamps.so
{ echo "== stamps single frame --cold"; timeout -k 10 180 python3 scripts/diag_stamps.py --cold 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
{ echo "== stamps single frame (warm)"; timeout -k 10 180 python3 scripts/diag_stamps.py 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
cat $OUT

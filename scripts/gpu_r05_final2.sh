# Round 5, last GPU call: the final check at HEAD (scripts/gpu_r05_check.sh: build --force on
# the box, the whole GPU suite, smoke, the driver's bench command, rocprofv3 traces, encoders,
# plain-C multi host), then session 24's A/B of the single-frame flat 8-bit path:
# uniform-random 2048x1536 one-frame launches (time_frame.py --random) and the config-2 frame
# command as a control, default vs noflat8 (MH_FLAT8=0), interleaved x 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_r05_check.sh > gpurun_out/r05_check3.txt 2>&1 || { tail -40 gpurun_out/r05_check3.txt; exit 1; }
echo "check done"
OUT=gpurun_out/r05_flat8_small_ab.txt
: > $OUT
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'])"; }
for rep in 1 2 3; do
  for v in default noflat8; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    timeout -k 10 120 python3 scripts/time_frame.py --random --tag $v 2>>gpurun_out/r05_flat8_small_ab.err | tail -1 >> $OUT || { echo "$v FAILED" >> $OUT; exit 1; }
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_flat8_small_ab.err) || { echo "$v frame FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
tail -30 gpurun_out/r05_check3.txt
cat $OUT

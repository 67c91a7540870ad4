# Kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) vs the runtime default, on the
# single-frame workload (cold regions) and the stamped launch (entry -> first header).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r04_kernarg_ab.txt
: > $OUT
for rep in 1 2 3; do
  for v in default devkernarg; do
    if [ $v = devkernarg ]; then export HIP_FORCE_DEV_KERNARG=1; else unset HIP_FORCE_DEV_KERNARG; fi
    for spec in frame:20:5 batch:20:5; do
      IFS=: read wl k w <<< "$spec"
      r=$(timeout -k 10 300 python bench.py --workload $wl --steps $k --warmup $w --no-extras --no-cpu-baseline 2>>gpurun_out/r04_kernarg_ab.err) || { echo "$v $wl FAILED" >> $OUT; exit 1; }
      echo "$v $wl:$k $r" | python3 -c "import sys,json; l=sys.stdin.read().split(' ',2); d=json.loads(l[2]); print(l[0], l[1], 'value', d['value'], 'warm', d.get('warm_value'), 'ungated', d.get('ungated_value'), 'kernel_us', d['roofline']['kernel_us_avg'])" >> $OUT
    done
  done
done
export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_stamps.so
for v in default devkernarg; do
  if [ $v = devkernarg ]; then export HIP_FORCE_DEV_KERNARG=1; else unset HIP_FORCE_DEV_KERNARG; fi
  { echo "== stamps single frame (warm) $v"; timeout -k 10 180 python3 scripts/diag_stamps.py 2>&1 | grep -v amdgpu.ids | grep -E "entry|hdr|launch|decomposition"; } >> $OUT || exit 1
done
cat $OUT

# A/B the experiment builds in ab on the batch + frame workloads.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/ab.txt
: > $OUT
for v in ${VARIANTS:-default $(ls ab | sed 's/^lib_//; s/\.so$//')}; do
  lib=$v; extra=""
  if [ "$lib" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$lib.so; fi
  for wl in ${WLS:-batch frame}; do
    r=$(timeout -k 10 300 python bench.py --workload $wl --steps ${STEPS:-50} --warmup 5 --no-extras --no-cpu-baseline $extra 2>>gpurun_out/ab.err) || { echo "$v $wl FAILED" >> $OUT; exit 1; }
    echo "$v $wl $r" | python -c "import sys,json; l=sys.stdin.read().split(' ',2); d=json.loads(l[2]); print(l[0], l[1], 'value', d['value'], 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'])" >> $OUT
  done
done
cat $OUT

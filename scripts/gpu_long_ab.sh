# Long launches (64-frame batch, 8192^2 frame): plain eager region vs a hipGraph behind the
# launch gate (MH_BENCH_LONG=graph), interleaved on one box -> gpurun_out/long_ab.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/long_ab.txt
for rep in 1 2 3; do
  for mode in eager graph graph_ungated; do
    for wl in batch tile8192; do
      k=256; [ $wl = tile8192 ] && k=512
      MH_BENCH_LONG=$mode timeout -k 10 300 python bench.py --workload $wl --steps $k --warmup $k --no-extras --no-cpu-baseline > gpurun_out/long_$mode_$wl.json 2> gpurun_out/long_err.txt || { tail gpurun_out/long_err.txt; exit 1; }
      python3 -c "import json,sys; d=json.load(open('gpurun_out/long_$mode_$wl.json')); r=d['roofline']; print('rep $rep $mode $wl', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', r['kernel_us_avg'], 'frac', r['frac'], d['config']['launch'])" >> gpurun_out/long_ab.txt
    done
  done
done
cat gpurun_out/long_ab.txt

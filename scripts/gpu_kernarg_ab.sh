# HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device memory) vs the runtime default, interleaved
# on one box: driver-shaped frame bench and the long launches (eager and graph) -> gpurun_out/kernarg_ab.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/kernarg_ab.txt
run() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline $BARGS > gpurun_out/ka.json 2> gpurun_out/ka_err.txt || { tail gpurun_out/ka_err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ka.json')); r=d['roofline']; print('$tag', d['config']['workload'][:8], d['value'], 'kernel_us', r['kernel_us_avg'], d['config']['launch'][:30])" >> gpurun_out/kernarg_ab.txt
}
for rep in 1 2; do
  for ka in default 1; do
    E=(); [ $ka = 1 ] && E=(HIP_FORCE_DEV_KERNARG=1)
    BARGS="--steps 20 --warmup 5" run "rep$rep ka=$ka frame" "${E[@]}" X=1 || exit 1
    BARGS="--workload batch --steps 256 --warmup 256" run "rep$rep ka=$ka batch-eager" "${E[@]}" MH_BENCH_LONG=eager || exit 1
    BARGS="--workload batch --steps 256 --warmup 256" run "rep$rep ka=$ka batch-graph" "${E[@]}" MH_BENCH_LONG=graph || exit 1
  done
done
cat gpurun_out/kernarg_ab.txt

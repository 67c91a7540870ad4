# Why are plain eager launches of the 64-frame batch slower than a graph replay? eager vs
# eager without the barrier bit (MH_BENCH_DIAG_RELAX=1) vs graph behind the gate, one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/long_ab2.txt
for rep in 1 2; do
  for mode in eager relax graph; do
    E=(MH_BENCH_LONG=eager); [ $mode = relax ] && E=(MH_BENCH_LONG=eager MH_BENCH_DIAG_RELAX=1); [ $mode = graph ] && E=(MH_BENCH_LONG=graph)
    env "${E[@]}" timeout -k 10 300 python bench.py --workload batch --steps 256 --warmup 256 --no-extras --no-cpu-baseline > gpurun_out/l2.json 2> gpurun_out/l2_err.txt || { tail gpurun_out/l2_err.txt; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/l2.json')); r=d['roofline']; print('rep $rep $mode', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', r['kernel_us_avg'], 'eager_med', r.get('eager_launch_us_median'))" >> gpurun_out/long_ab2.txt
  done
done
cat gpurun_out/long_ab2.txt

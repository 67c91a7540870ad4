# Driver-shaped bench (20 steps, 5 warm-up, frame workload): graph replay vs eager
# launches behind the launch gate, interleaved, 3 reps each.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/gate_graph_ab.txt
for rep in 1 2 3; do
  for mode in graph eager; do
    extra=""; [ $mode = eager ] && extra="--no-graph"
    r=$(timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline $extra 2>>gpurun_out/gate_graph_ab.err) || { echo "$mode FAILED"; exit 1; }
    echo "$r" | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$mode', 'value', d['value'], 'ms_per_step', d['ms_per_step'], 'region_ms', d['gpu_region_ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'ungated', d.get('ungated_value'))" >> gpurun_out/gate_graph_ab.txt
  done
done
cat gpurun_out/gate_graph_ab.txt

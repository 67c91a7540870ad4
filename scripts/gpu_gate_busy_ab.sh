# Driver-shaped bench (20 steps) under the env settings in KINDS (e.g. MH_BENCH_GATE_KIND=busy:
# CUs issuing ALU work while the gate is closed), interleaved, 3 reps.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/gate_busy_ab.txt
for rep in 1 2 3; do
  for kind in ${KINDS:-kernel busy}; do
    r=$(env $kind timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/gate_busy_ab.err) || { echo "$kind FAILED"; exit 1; }
    echo "$r" | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$kind'.split('=')[-1], 'value', d['value'], 'ms_per_step', d['ms_per_step'], 'region_ms', d['gpu_region_ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'])" >> gpurun_out/gate_busy_ab.txt
  done
done
cat gpurun_out/gate_busy_ab.txt

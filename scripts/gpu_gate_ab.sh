# Launch gate A/B: polling kernel vs hipStreamWaitValue32, the driver's 20-step command.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/gate_ab.txt
for rep in 1 2 3; do
  for kind in kernel wait; do
    MH_BENCH_GATE_KIND=$kind timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/gate_$kind.json 2> gpurun_out/gate_$kind.err || { echo "$kind failed"; tail gpurun_out/gate_$kind.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/gate_$kind.json'));r=d['roofline'];print('$kind', 'value', d['value'], 'ms', d['ms_per_step'], 'region', r['region_us_per_launch'], 'kernel', r['kernel_us_avg'], 'ungated', d['ungated_ms_per_step'])" >> gpurun_out/gate_ab.txt
  done
done
cat gpurun_out/gate_ab.txt

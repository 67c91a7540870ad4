# The driver's bench command (--steps 20 --warmup 5), repeated: headline spread.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/b20_rep.txt
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/b20_$i.json 2> gpurun_out/b20_$i.err || { tail gpurun_out/b20_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/b20_$i.json'));print('value',d['value'],'ms',d['ms_per_step'],'ungated',d.get('ungated_value'),d.get('ungated_ms_per_step'),'kernel_us',d['roofline']['kernel_us_avg'],'read_frac',d['roofline'].get('read_frac'))" >> gpurun_out/b20_rep.txt
done
cat gpurun_out/b20_rep.txt
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b20.json 2> gpurun_out/b20.err || { tail gpurun_out/b20.err; exit 1; }
cat gpurun_out/b20.json

# Two ranks on the box's one GPU over gloo (MH_BENCH_BACKEND=gloo): the N > 1 bench
# path end to end (header broadcast, device tables, parity guard on both ranks, gated
# regions, config-4 and config-5 extras). The driver's 8-GPU runs use RCCL.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
MH_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 \
  > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2_gloo.err || { tail -30 gpurun_out/bench_n2_gloo.err; exit 1; }
python3 -c "
import json
d = json.loads(open('gpurun_out/bench_n2_gloo.json').read().strip().splitlines()[-1])
print('n_gpus', d['n_gpus'], 'value', d['value'], 'ms_per_step', d['ms_per_step'], d['config'].get('launch'))
print('extras', sorted(d.get('extras', {}).keys()))
print('ranks_verified', d.get('ranks_verified'), 'rank_devices', d.get('rank_devices'))
"

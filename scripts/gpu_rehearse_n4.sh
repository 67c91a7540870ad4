# Four ranks on the box's one GPU over gloo (MH_BENCH_BACKEND=gloo): the N > 1 bench path with more
# than two ranks (header broadcast, device tables, parity guard on every rank, gated regions,
# config-4 and config-5 extras, rank_devices). The driver's multi-GPU runs use RCCL.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
MH_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29527 bench.py --gpus 4 --steps 20 --warmup 5 \
  > gpurun_out/bench_n4_gloo.json 2> gpurun_out/bench_n4_gloo.err || { tail -30 gpurun_out/bench_n4_gloo.err; exit 1; }
python3 -c "
import json
d = json.loads(open('gpurun_out/bench_n4_gloo.json').read().strip().splitlines()[-1])
print('n_gpus', d['n_gpus'], 'value', d['value'], 'ms_per_step', d['ms_per_step'], d['config'].get('launch'))
print('extras', sorted(d.get('extras', {}).keys()))
print('ranks_verified', d.get('ranks_verified'), 'rank_devices', d.get('rank_devices'))
"

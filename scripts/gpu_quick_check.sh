# GPU tests (selected with K, default all), then the default bench line at the
# driver's 20 steps and at 200 (fail-fast).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/bench20.json 2> gpurun_out/bench20.err || { tail gpurun_out/bench20.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench20.json')); print('20 steps', d['value'], d['ms_per_step'], d['config']['launch'], d['roofline']['kernel_us_avg'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/bench20b.json 2>> gpurun_out/bench20.err || { tail gpurun_out/bench20.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench20b.json')); print('20 steps', d['value'], d['ms_per_step'], d['config']['launch'], d['roofline']['kernel_us_avg'])"

# Long-launch timed region A/B: all K/16 graph replays queued behind the launch gate
# (MH_BENCH_LONG=graph) vs only the first (window, the default), unprofiled and under
# rocprofv3 --kernel-trace (timed_steady from the trace markers).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/window_ab.txt
: > $OUT
for rep in 1 2; do
  for m in graph window; do
    for wl in batch tile8192; do
      r=$(MH_BENCH_LONG=$m timeout -k 10 300 python bench.py --workload $wl --steps 256 --warmup 64 --no-extras --no-cpu-baseline 2>>gpurun_out/window_ab.err) || exit 1
      echo "$r" | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$m $wl value', d['value'], 'kernel_us', r['kernel_us_avg'], 'region_us', r['region_us_per_launch'], 'graph_us', r['graph_us_per_launch'])" >> $OUT
    done
  done
done
for m in graph window; do
  for wl in batch tile8192; do
    rm -rf gpurun_out/wprof_${m}_$wl
    MH_BENCH_LONG=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wprof_${m}_$wl -o run -- \
      python3 bench.py --workload $wl --steps 256 --warmup 64 --no-extras --no-cpu-baseline > gpurun_out/wprof_${m}_$wl.json 2>gpurun_out/wprof.err || exit 1
    k=$(python3 -c "import json; print(json.loads(open('gpurun_out/wprof_${m}_$wl.json').read().strip().splitlines()[-1])['roofline']['kernel_us_avg'])")
    echo "== profiled $m $wl: line kernel_us_avg $k" >> $OUT
    python3 scripts/ktrace_summary.py gpurun_out/wprof_${m}_$wl 256 16 >> $OUT || exit 1
  done
done
cat $OUT

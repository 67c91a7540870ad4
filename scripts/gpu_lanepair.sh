# Lane-pair variant: parity tests, then an interleaved A/B against the default
# single-frame kernel (the driver's bench command shape, kernel time from HIP events).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lane_pairs.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_lp.log 2>&1 || { tail -40 gpurun_out/pytest_lp.log; exit 1; }
tail -3 gpurun_out/pytest_lp.log
OUT=gpurun_out/lp_ab.txt
: > $OUT
for rep in 1 2; do
  for fl in 0 2; do
    MH_BENCH_DECODE_FLAGS=$fl timeout -k 10 300 python bench.py --workload frame --steps 200 --warmup 20 --no-extras --no-cpu-baseline > gpurun_out/lp_$fl.json 2>>gpurun_out/lp_ab.err || { echo "flags $fl FAILED" >> $OUT; tail gpurun_out/lp_ab.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/lp_$fl.json'));r=d['roofline'];print('rep $rep flags $fl', 'value', d['value'], 'kernel_us', r['kernel_us_avg'], 'frac', r['frac'], 'verified', d['frames_verified'])" >> $OUT
  done
done
cat $OUT
rm -rf gpurun_out/prof_lp
MH_BENCH_DECODE_FLAGS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_lp -o run -- python3 bench.py --workload frame --steps 200 --warmup 20 --no-extras --no-cpu-baseline > gpurun_out/lp_prof.json 2> gpurun_out/lp_prof.err || { tail gpurun_out/lp_prof.err; exit 1; }
python3 scripts/ktrace_summary.py gpurun_out/prof_lp 200 | tee gpurun_out/lp_ktrace.txt

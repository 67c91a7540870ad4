# CPU frame decoder A/B (default library vs ab/lib_cpu_static.so, interleaved), then the
# batch and tile8192 kernel traces re-run (profiles/r03_v11_cpu_row_counter_negative_ab.txt,
# profiles/r03_ktrace_summary.txt)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/cpu_ab.txt
for rep in 1 2 3; do
  for v in counter static; do
    if [ $v = static ]; then export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_cpu_static.so; else unset MH_LIB; fi
    echo "== $v" >> gpurun_out/cpu_ab.txt
    timeout -k 10 120 python -u scripts/cpu_frame_decoder.py 20 >> gpurun_out/cpu_ab.txt 2>&1 || exit 1
  done
done
unset MH_LIB
cat gpurun_out/cpu_ab.txt
: > gpurun_out/ktrace_summary2.txt
for spec in batch:256:256 tile8192:512:512; do
  IFS=: read wl k w <<< "$spec"
  rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof2_$wl
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof2_$wl -o run -- python3 bench.py --workload $wl --steps $k --warmup $w --no-extras --no-cpu-baseline > gpurun_out/bench_prof2_$wl.json 2> gpurun_out/bench_prof2_$wl.err || { tail gpurun_out/bench_prof2_$wl.err; exit 1; }
  u=$(python3 -c "import json;print(json.load(open('gpurun_out/bench_prof2_$wl.json'))['roofline'].get('kernel_us_steady_unit') or 1)")
  { echo "== bench.py --workload $wl --steps $k --warmup $w (profiled line: roofline.kernel_us_avg $(python3 -c "import json;print(json.load(open('gpurun_out/bench_prof2_$wl.json'))['roofline']['kernel_us_avg'])"), steady unit $u)"; python3 scripts/ktrace_summary.py gpurun_out/prof2_$wl $k $u; } >> gpurun_out/ktrace_summary2.txt
done
cat gpurun_out/ktrace_summary2.txt

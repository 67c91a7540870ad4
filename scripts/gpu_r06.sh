# Round-6 GPU steps, one parameterised script (fail-fast; every GPU step under its own
# timeout; the call ends at the first failure):
#   bash scripts/gpu_r06.sh <step> [<step> ...]
# steps:
#   forensic        round 5's spilled batch-loop build vs the kept one (ab/lib_spill.so,
#                   ab/lib_fix.so): scripts/forensic_spill.py on both   -> gpurun_out/forensic_*.log
#   forensic:<lib>  the same for ab/lib_<lib>.so only
#   tests           the whole GPU suite                                 -> gpurun_out/pytest_gpu.log
#   smoke           __graft_entry__.smoke()
#   bench           the driver's bench command                          -> gpurun_out/bench.json
#   ab:<w>:<reps>:<libs>   interleaved bench --workload <w> over default + ab/lib_<x>.so (comma list)
#   traces          rocprofv3 kernel traces of each workload's bench command
#   pmc:<wl>        counter passes (scripts/gpu_profile.sh groups) for one workload
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for step in "$@"; do
  echo "== step $step $(date +%T)"
  case "$step" in
    forensic|forensic:*)
      libs=${step#forensic}; libs=${libs#:}; [ -z "$libs" ] && libs="spill fix"
      for l in $libs; do
        MH_LIB=$PWD/ab/lib_$l.so timeout -k 10 300 python -u scripts/forensic_spill.py --cases ${FORENSIC_CASES:-random8192,flatmulti,noesc,general} > gpurun_out/forensic_$l.log 2>&1 || { tail -30 gpurun_out/forensic_$l.log; exit 1; }
        grep -v "^    " gpurun_out/forensic_$l.log
      done ;;
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
      tail -1 gpurun_out/pytest_gpu.log ;;
    tests:*)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "${step#tests:}" > gpurun_out/pytest_gpu_k.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_k.log; exit 1; }
      tail -1 gpurun_out/pytest_gpu_k.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
      tail -1 gpurun_out/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
      cat gpurun_out/bench.json ;;
    ab:*)
      IFS=: read _ wl reps libs <<< "$step"
      out=gpurun_out/ab_$wl.txt
      for r in $(seq $reps); do
        for l in default ${libs//,/ }; do
          if [ $l = default ]; then env=""; else env="MH_LIB=$PWD/ab/lib_$l.so"; fi
          env $env timeout -k 10 300 python bench.py --workload $wl --steps 200 --warmup 50 --no-extras --no-cpu-baseline > gpurun_out/ab_one.json 2> gpurun_out/ab_one.err || { tail gpurun_out/ab_one.err; exit 1; }
          python3 -c "import json;d=json.load(open('gpurun_out/ab_one.json'));r=d['roofline'];print('$l', '$wl', 'value', d['value'], 'kernel_us', r['kernel_us_avg'], 'frac', round(r['frac'],4))" | tee -a $out
        done
      done ;;
    traces)
      : > gpurun_out/ktrace_summary.txt
      for spec in frame:20:5 batch:256:256 tile8192:512:512 tile8192_random:512:512; do
        IFS=: read wl k w <<< "$spec"
        rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_$wl
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$wl -o run -- python3 bench.py --workload $wl --steps $k --warmup $w --no-extras --no-cpu-baseline > gpurun_out/bench_prof_$wl.json 2> gpurun_out/bench_prof_$wl.err || { tail gpurun_out/bench_prof_$wl.err; exit 1; }
        u=$(python3 -c "import json;print(json.load(open('gpurun_out/bench_prof_$wl.json'))['roofline'].get('kernel_us_steady_unit') or 1)")
        { echo "== bench.py --workload $wl --steps $k --warmup $w (profiled line: roofline.kernel_us_avg $(python3 -c "import json;print(json.load(open('gpurun_out/bench_prof_$wl.json'))['roofline']['kernel_us_avg'])"), steady unit $u)"; python3 scripts/ktrace_summary.py gpurun_out/prof_$wl $k $u; } >> gpurun_out/ktrace_summary.txt
      done
      cat gpurun_out/ktrace_summary.txt ;;
    pmc:*)
      IFS=: read _ wl kern groups <<< "$step"
      rm -rf gpurun_out/pmc_$wl
      WL=$wl OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$wl PMC_GROUPS="$groups" bash scripts/gpu_profile.sh || exit 1
      { echo "== $wl ($kern)"; python3 scripts/pmc_summary.py gpurun_out/pmc_$wl $kern 2; } | tee -a gpurun_out/pmc_kernels.txt ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done

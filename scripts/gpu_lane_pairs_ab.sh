# Lane-pair cursor (MH_FLAG_LANE_PAIRS): parity tests, bench A/B
# against the default single-frame kernel on config 2, and one PMC pass per flavour
# (instructions per wave -> per decode step, compared with scripts/sim_lane_groups_sync.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_lane_pairs.py tests/test_gpu_stress.py tests/test_gpu_decode.py::test_any_order_run_of_frames \
  > gpurun_out/lp_tests.log 2>&1 || { tail -40 gpurun_out/lp_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/lp_tests.log | tail -2
OUT=gpurun_out/lp_ab.txt
: > $OUT
# runs: <library>:<decode flags>; VARIANTS from ab/ (e.g. lpv1:2) join the default ones
RUNS="default:0 default:2 ${VARIANTS:-}"
for rep in 1 2; do
  for run in $RUNS; do
    IFS=: read v fl <<< "$run"
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(MH_BENCH_DECODE_FLAGS=$fl timeout -k 10 300 python bench.py --workload frame --steps 200 --warmup 20 --no-extras --no-cpu-baseline 2>>gpurun_out/lp_ab.err) || exit 1
    echo "$r" | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v flags $fl', 'value', d['value'], 'kernel_us', r['kernel_us_avg'], 'region_us', r['region_us_per_launch'])" >> $OUT
  done
done
unset MH_LIB
cat $OUT
for run in $RUNS; do
  IFS=: read v fl <<< "$run"
  if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
  rm -rf gpurun_out/lp_pmc_${v}_$fl
  MH_BENCH_DECODE_FLAGS=$fl timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH GRBM_GUI_ACTIVE \
    --output-format csv -d gpurun_out/lp_pmc_${v}_$fl/pmc1 -o run -- python3 bench.py --workload frame --steps 10 --warmup 2 --no-extras --no-cpu-baseline > gpurun_out/lp_pmc_${v}_$fl.log 2>&1 || { tail -5 gpurun_out/lp_pmc_${v}_$fl.log; exit 1; }
  k=mh_decode_small_kernel; [ $fl = 2 ] && k=mh_decode_lanepair_kernel
  echo "== $v flags $fl ($k)"; python3 scripts/pmc_summary.py gpurun_out/lp_pmc_${v}_$fl $k 2
done

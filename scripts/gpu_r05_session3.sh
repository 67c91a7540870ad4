# Round 5, GPU session 3: the whole GPU suite on this tree; the batched encoder A/B
# (default = this tree: tile tails kept by the split; encr04 = round-4 encoder; enc256 =
# tile tails + 256-block batch tiles) with HIP-event timing and HBM traffic per variant;
# rocprofv3 kernel traces of batch / tile8192 / tile8192_random at this HEAD (VERDICT r04
# item 2).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r05_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r05_pytest_gpu.log
OUT=gpurun_out/r05_enc_ab.txt
: > $OUT
VARIANTS="encr04 enc256"
for rep in 1 2 3; do
  for v in default $VARIANTS; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    timeout -k 10 120 python3 scripts/enc_batch_profile.py 64 8 2>&1 | grep "^batch" | tail -1 | sed "s/^/$v /" >> $OUT || exit 1
  done
done
echo "enc timing done"
for v in default $VARIANTS; do
  if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
  for ctr in FETCH_SIZE WRITE_SIZE; do
    d=gpurun_out/pmc_enc_${v}_$ctr
    rm -rf $d
    timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $GRAFT_REPO_ROOT/$d/pmc -o run -- python3 scripts/enc_batch_profile.py 64 2 > $d.log 2>&1 || { echo "pmc $v $ctr failed"; tail -5 $d.log; exit 1; }
  done
  alg=$(grep -o "alg_bytes [0-9]*" gpurun_out/pmc_enc_${v}_FETCH_SIZE.log | head -1 | cut -d" " -f2)
  { echo "== traffic $v"; python3 scripts/enc_batch_pmc.py gpurun_out/pmc_enc_${v}_FETCH_SIZE gpurun_out/pmc_enc_${v}_WRITE_SIZE --alg $alg; } >> $OUT 2>&1
  echo "traffic $v done"
done
unset MH_LIB
cat $OUT
: > gpurun_out/r05_ktrace_summary.txt
for spec in frame:20:5 batch:256:256 tile8192:512:512 tile8192_random:512:512; do
  IFS=: read wl k w <<< "$spec"
  rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_$wl
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$wl -o run -- python3 bench.py --workload $wl --steps $k --warmup $w --no-extras --no-cpu-baseline > gpurun_out/bench_prof_$wl.json 2> gpurun_out/bench_prof_$wl.err || { tail gpurun_out/bench_prof_$wl.err; exit 1; }
  u=$(python3 -c "import json;print(json.load(open('gpurun_out/bench_prof_$wl.json'))['roofline'].get('kernel_us_steady_unit') or 1)")
  { echo "== bench.py --workload $wl --steps $k --warmup $w (profiled line: roofline.kernel_us_avg $(python3 -c "import json;print(json.load(open('gpurun_out/bench_prof_$wl.json'))['roofline']['kernel_us_avg'])"), steady unit $u)"; python3 scripts/ktrace_summary.py gpurun_out/prof_$wl $k $u; } >> gpurun_out/r05_ktrace_summary.txt
  echo "ktrace $wl done"
done
cat gpurun_out/r05_ktrace_summary.txt

# Round 5, GPU session 4: batched encoder at 256-block tiles (default) vs 128 / 512:
# encoder GPU tests, HIP-event timing (3 reps interleaved), a kernel trace per variant
# (per-kernel split), HBM traffic of enc512.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode_batch.py tests/test_gpu_encode.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05_pytest_enc.log 2>&1 || { tail -40 gpurun_out/r05_pytest_enc.log; exit 1; }
tail -1 gpurun_out/r05_pytest_enc.log
OUT=gpurun_out/r05_enc_ab2.txt
: > $OUT
VARIANTS="enc128 enc512"
for rep in 1 2 3; do
  for v in default $VARIANTS; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    timeout -k 10 120 python3 scripts/enc_batch_profile.py 64 8 2>&1 | grep "^batch" | tail -1 | sed "s/^/$v /" >> $OUT || exit 1
  done
done
for v in default $VARIANTS; do
  if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
  rm -rf gpurun_out/prof_ab_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_ab_$v -o run -- python3 scripts/enc_batch_profile.py 64 8 > gpurun_out/prof_ab_$v.log 2>&1 || { tail gpurun_out/prof_ab_$v.log; exit 1; }
  python3 - "$v" <<'PY' >> $OUT
import csv, sys
v = sys.argv[1]
for r in sorted(csv.DictReader(open(f"gpurun_out/prof_ab_{v}/run_kernel_stats.csv")), key=lambda r: -float(r["TotalDurationNs"]))[:3]:
    print(f"{v} kernel {float(r['AverageNs']) / 1e3:9.2f} us  x{r['Calls']:>4}  {r['Name'][:70]}")
PY
done
for v in enc512; do
  export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so
  for ctr in FETCH_SIZE WRITE_SIZE; do
    d=gpurun_out/pmc_enc_${v}_$ctr
    rm -rf $d
    timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $GRAFT_REPO_ROOT/$d/pmc -o run -- python3 scripts/enc_batch_profile.py 64 2 > $d.log 2>&1 || { echo "pmc $v $ctr failed"; tail -5 $d.log; exit 1; }
  done
  alg=$(grep -o "alg_bytes [0-9]*" gpurun_out/pmc_enc_${v}_FETCH_SIZE.log | head -1 | cut -d" " -f2)
  { echo "== traffic $v"; python3 scripts/enc_batch_pmc.py gpurun_out/pmc_enc_${v}_FETCH_SIZE gpurun_out/pmc_enc_${v}_WRITE_SIZE --alg $alg; } >> $OUT 2>&1
done
unset MH_LIB
cat $OUT

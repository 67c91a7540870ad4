# Round 5, GPU session 9: tiled split without dead per-row stores (encoder GPU tests, then
# default vs encprev = the encoder before this change, 3 reps interleaved + per-kernel trace).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode_batch.py tests/test_gpu_encode.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05_pytest_enc2.log 2>&1 || { tail -40 gpurun_out/r05_pytest_enc2.log; exit 1; }
tail -1 gpurun_out/r05_pytest_enc2.log
OUT=gpurun_out/r05_enc_ab3.txt
: > $OUT
VARIANTS="encprev"
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
unset MH_LIB
cat $OUT

# Encoder A/B: parity (GPU encoder tests), async rate per variant, tree kernel time and
# its phase clocks (stamps builds).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_tables.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_enc.log 2>&1 || { tail -30 gpurun_out/pytest_enc.log; exit 1; }
tail -1 gpurun_out/pytest_enc.log
: > gpurun_out/enc_ab.txt
for rep in 1 2; do
for v in default ${ENC_VARIANTS:-tree_bsearch}; do
  if [ $v = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
  rm -rf gpurun_out/prof_enc_$v
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_enc_$v -o run -- python3 scripts/enc_profile.py 64 > gpurun_out/enc_$v.log 2>&1 || { tail gpurun_out/enc_$v.log; exit 1; }
  timeout -k 10 120 python3 scripts/enc_profile.py 256 > gpurun_out/enc_plain_$v.log 2>&1 || { tail gpurun_out/enc_plain_$v.log; exit 1; }
  { echo "== $v: unprofiled $(grep 'async encode' gpurun_out/enc_plain_$v.log)"; python3 - $v <<'PY'
import csv, sys
v = sys.argv[1]
for r in sorted(csv.DictReader(open(f"gpurun_out/prof_enc_{v}/run_kernel_stats.csv")), key=lambda r: -float(r["AverageNs"])):
    print(f"   {float(r['AverageNs']) / 1e3:8.2f} us  x{r['Calls']:>4}  {r['Name'][:70]}")
PY
  } >> gpurun_out/enc_ab.txt
done
done
for v in ${STAMP_VARIANTS:-stamps stamps_bsearch}; do
  export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so
  echo "== $v" >> gpurun_out/enc_ab.txt
  timeout -k 10 120 python3 scripts/enc_profile.py 16 stamps >> gpurun_out/enc_ab.txt 2>&1 || { echo "stamps $v failed"; exit 1; }
done
cat gpurun_out/enc_ab.txt

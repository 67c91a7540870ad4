# Batched encoder A/B: the encoder GPU tests on the default library, then variants from
# ab/ (VARIANTS) interleaved with it (scripts/enc_batch_profile.py 64 8, HIP events), one
# rocprofv3 kernel trace each (per-kernel split), then PMC passes on the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode_batch.py tests/test_gpu_encode.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_enc.log 2>&1 || { tail -30 gpurun_out/pytest_enc.log; exit 1; }
tail -1 gpurun_out/pytest_enc.log
: > gpurun_out/enc_batch_ab.txt
for rep in 1 2; do
  for v in default $VARIANTS; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    timeout -k 10 120 python3 scripts/enc_batch_profile.py 64 8 2>&1 | grep "^batch" | tail -1 | sed "s/^/$v /" >> gpurun_out/enc_batch_ab.txt || exit 1
  done
done
for v in default $VARIANTS; do
  if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
  rm -rf gpurun_out/prof_ab_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_ab_$v -o run -- python3 scripts/enc_batch_profile.py 64 8 > gpurun_out/prof_ab_$v.log 2>&1 || { tail gpurun_out/prof_ab_$v.log; exit 1; }
  python3 - "$v" <<'PY' >> gpurun_out/enc_batch_ab.txt
import csv, sys
v = sys.argv[1]
for r in sorted(csv.DictReader(open(f"gpurun_out/prof_ab_{v}/run_kernel_stats.csv")), key=lambda r: -float(r["TotalDurationNs"]))[:3]:
    print(f"{v} kernel {float(r['AverageNs']) / 1e3:9.2f} us  x{r['Calls']:>4}  {r['Name'][:70]}")
PY
done
unset MH_LIB
cat gpurun_out/enc_batch_ab.txt
rm -rf gpurun_out/pmc_enc_*
for ctr in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_BUSY_CYCLES"; do
  d=gpurun_out/pmc_enc_${ctr%% *}
  timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $GRAFT_REPO_ROOT/$d -o run -- python3 scripts/enc_batch_profile.py 64 2 > $d.log 2>&1 || { echo "pmc $ctr failed"; tail -5 $d.log; exit 1; }
done
python3 scripts/enc_batch_pmc.py gpurun_out/pmc_enc_* --alg $(grep -o "alg_bytes [0-9]*" gpurun_out/pmc_enc_FETCH_SIZE.log | head -1 | cut -d" " -f2) | tee gpurun_out/enc_batch_pmc.txt

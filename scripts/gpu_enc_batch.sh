# Batched encoder: its GPU tests, a rocprofv3 kernel trace of 8 calls of 64 frames, then
# PMC passes (one counter group per run): HBM bytes and SQ counters per kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode_batch.py tests/test_gpu_encode.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_enc.log 2>&1 || { tail -30 gpurun_out/pytest_enc.log; exit 1; }
tail -1 gpurun_out/pytest_enc.log
rm -rf gpurun_out/prof_encb
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_encb -o run -- python3 scripts/enc_batch_profile.py 64 8 > gpurun_out/enc_batch.log 2>&1 || { tail gpurun_out/enc_batch.log; exit 1; }
grep batch gpurun_out/enc_batch.log
python3 - <<'PY'
import csv
for r in sorted(csv.DictReader(open("gpurun_out/prof_encb/run_kernel_stats.csv")), key=lambda r: -float(r["TotalDurationNs"]))[:4]:
    print(f"{float(r['AverageNs']) / 1e3:9.2f} us  x{r['Calls']:>4}  {r['Name'][:90]}")
PY
rm -rf gpurun_out/pmc_enc_*
for ctr in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_BUSY_CYCLES"; do
  d=gpurun_out/pmc_enc_${ctr%% *}
  timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $GRAFT_REPO_ROOT/$d -o run -- python3 scripts/enc_batch_profile.py 64 2 > $d.log 2>&1 || { echo "pmc $ctr failed"; tail -5 $d.log; exit 1; }
done
python3 scripts/enc_batch_pmc.py gpurun_out/pmc_enc_* --alg $(grep -o "alg_bytes [0-9]*" gpurun_out/enc_batch.log | head -1 | cut -d" " -f2) | tee gpurun_out/enc_batch_pmc.txt

cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_encode_batch.py -v --timeout 150 --timeout-method thread > gpurun_out/pytest_enc.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|assert" gpurun_out/pytest_enc.log | tail -40
exit $rc

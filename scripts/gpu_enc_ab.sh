# Encoder A/B: HEAD vs a variant library (VARIANT, from ab/), the GPU encoder tests on
# HEAD, then async back-to-back time per frame (scripts/enc_profile.py), interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_encode.py \
  > gpurun_out/enc_tests.log 2>&1 || { tail -30 gpurun_out/enc_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/enc_tests.log | tail -1
: > gpurun_out/enc_ab.txt
for rep in 1 2 3; do
  for v in default ${VARIANT:-}; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    echo "== $v" >> gpurun_out/enc_ab.txt
    timeout -k 10 120 python3 scripts/enc_profile.py 64 2>&1 | grep -v amdgpu.ids >> gpurun_out/enc_ab.txt || exit 1
  done
done
unset MH_LIB
cat gpurun_out/enc_ab.txt

# Encoder: parity, tree phase stamps, then per-kernel times of the default build and
# of each variant in ab (rocprofv3 kernel trace).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_encode.py > gpurun_out/enc_tests.log 2>&1 || { tail -30 gpurun_out/enc_tests.log; exit 1; }
tail -1 gpurun_out/enc_tests.log
if [ -f ab/lib_treestamps.so ]; then
  MH_LIB=$GRAFT_REPO_ROOT/ab/lib_treestamps.so timeout -k 10 120 python3 scripts/enc_profile.py 16 stamps 2>&1 | grep -v amdgpu.ids || exit 1
fi
for v in default ${VARIANTS:-}; do
  if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/encab_$v -o enc -- python3 scripts/enc_profile.py 64 > gpurun_out/encab_$v.log 2>&1 || exit 1
  echo "== $v: $(grep async gpurun_out/encab_$v.log)"
  python3 - "$v" <<'PY' || exit 1
import glob, sqlite3, sys
c = sqlite3.connect(glob.glob(f"gpurun_out/encab_{sys.argv[1]}/*.db")[0])
for name, n, avg in c.execute("select name, count(*), avg(end-start)/1000.0 from kernels group by name order by 3 desc"):
    print(f"   {avg:8.2f} us  x{n}  {name[:60]}")
PY
done

# Round 5, GPU session 2: where did round 4's batch-kernel time go?
#  (a) the new per-flavour multi-tile test, then
#  (b) a 2 x 2 of MEASUREMENT METHOD x KERNEL CODE on one box, interleaved: the round-3
#      tree's own bench.py (warm: a region re-decodes the same resident launch) and this
#      tree's bench.py (cold: a 1 GiB flush and launches no earlier region touched), each
#      with the round-3 library (ab/r03tree, built from f433465) and this tree's library;
#  (c) the code bisect under this bench.py: r03 (f433465), c8397 (8397e6d: one loop with a
#      per-tile flavour switch), head (r04 HEAD), split (this tree: one loop instantiation
#      per flavour again), then one PMC pass per variant on the batch.
set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05_pytest_decode.log 2>&1 || { tail -40 gpurun_out/r05_pytest_decode.log; exit 1; }
tail -1 gpurun_out/r05_pytest_decode.log
OUT=gpurun_out/r05_method_ab.txt
: > $OUT
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'], 'warm', d.get('warm_value'))"; }
for rep in 1 2; do
  for bench in r03 r05; do
    for lib in r03 r05; do
      # the round-3 kernels: the r03 tree's own library under its own bench.py; under this
      # bench.py (whose package binds symbols added since) ab/lib_r03.so = f433465's
      # mh_decode.hip linked with this tree's other sources -- the same decode kernels
      if [ $lib = r03 ]; then
        if [ $bench = r03 ]; then L=$ROOT/ab/r03tree/metalhuffman_amd/libmetalhuffman_amd.so; else L=$ROOT/ab/lib_r03.so; fi
      else L=$ROOT/metalhuffman_amd/libmetalhuffman_amd.so; fi
      if [ $bench = r03 ]; then D=$ROOT/ab/r03tree; else D=$ROOT; fi
      for wl in batch tile8192 tile8192_random; do
        r=$(cd $D && MH_LIB=$L timeout -k 10 150 python bench.py --workload $wl --steps 64 --warmup 16 --no-extras --no-cpu-baseline 2>>$ROOT/gpurun_out/r05_method_ab.err) || { echo "bench_$bench lib_$lib $wl FAILED" >> $OUT; exit 1; }
        echo "bench_$bench lib_$lib $wl $(echo "$r" | line)" >> $OUT
      done
      echo "rep $rep bench $bench lib $lib done"
    done
  done
done
cat $OUT
PMC=1 bash scripts/gpu_r05_bisect.sh

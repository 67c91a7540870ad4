# Round 5, GPU session 14: the batch kernel's row-store policy under the cold method (round 3
# chose nt = 2 on warm regions): default (nt) vs write-through nt sc1 (18) vs the default
# policy (0); batch and 8192^2 (mirror tile and random), 64-step regions, interleaved x 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_batch_store_ab.txt
: > $OUT
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'])"; }
for rep in 1 2 3; do
  for v in default bst18 bst0; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    for wl in batch tile8192 tile8192_random; do
      r=$(timeout -k 10 150 python bench.py --workload $wl --steps 64 --warmup 16 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_batch_store_ab.err) || { echo "$v $wl FAILED" >> $OUT; exit 1; }
      echo "$v $wl $(echo "$r" | line)" >> $OUT
    done
  done
  echo "rep $rep done"
done
cat $OUT

# Round 5, GPU session 26: PMC traffic at HEAD (scripts/gpu_traffic.sh: FETCH_SIZE / WRITE_SIZE
# per workload, the flat 8-bit path included), then where the flat path's time goes: 8 uniform-
# random 2048x1536 frames per launch (6,144 tiles, the batch kernel's flat path) timed by
# time_frame.py for the default (nt stores), plain stores (f8aux0), write-through (f8aux18) and
# every row store dropped (f8drop, reads only; output wrong on purpose), interleaved x 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_traffic.sh > gpurun_out/r05_traffic_run.txt 2>&1 || { tail -30 gpurun_out/r05_traffic_run.txt; exit 1; }
echo "traffic done"
OUT=gpurun_out/r05_flat8_stores_ab.txt
: > $OUT
for rep in 1 2 3; do
  for v in default f8aux0 f8aux18 f8drop; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    timeout -k 10 120 python3 scripts/time_frame.py --random --batch 8 --k 100 --tag $v 2>>gpurun_out/r05_flat8_stores_ab.err | tail -1 >> $OUT || { echo "$v FAILED" >> $OUT; exit 1; }
  done
  echo "rep $rep done"
done
cat gpurun_out/traffic.json
cat $OUT

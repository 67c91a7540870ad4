# Single-frame kernel A/B: the default library vs ab/lib_$V.so (MH_LIB), interleaved, driver-shaped
# bench (20 steps) -> gpurun_out/frame_ab_$V.txt.   V=tlbpf bash scripts/gpu_frame_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/frame_ab_$V.txt
: > $OUT
for rep in 1 2 3; do
  for lib in default $V; do
    E=(X=1); [ $lib != default ] && E=(MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$lib.so)
    env "${E[@]}" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/fab.json 2> gpurun_out/fab_err.txt || { tail gpurun_out/fab_err.txt; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/fab.json')); r=d['roofline']; print('rep $rep $lib', d['value'], 'kernel_us', r['kernel_us_avg'], 'verified', d['frames_verified'])" >> $OUT
  done
done
cat $OUT

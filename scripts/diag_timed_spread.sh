cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for spin in auto spin; do for s in 25; do
MH_BENCH_SYNC=$spin MH_BENCH_DIAG_REPEAT=12 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > /dev/null 2> gpurun_out/d_$spin$s.err || exit 1
echo "spin=$spin: $(grep diag gpurun_out/d_$spin$s.err | awk '{print $3}' | tr '\n' ' ')"
done; done

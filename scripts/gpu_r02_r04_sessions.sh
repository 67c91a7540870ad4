# Rounds 2-4: one-off GPU A/B and check sessions (folded in round 6)
# Each former one-off GPU session script is one case below, verbatim (the profiles/ record each produced
# is named in its header comment). Run one as:  bash scripts/gpu_r02_r04_sessions.sh <name>
# names: gpu_bench20 gpu_grid_ab gpu_kernarg_ab gpu_long_ab2 gpu_long_ab gpu_r04_ab2 gpu_r04_ab3 gpu_r04_ab4 gpu_r04_check gpu_r04_frame_stamps gpu_r04_kernarg_ab gpu_r04_tile_ab gpu_window_ab
set -o pipefail
case "$1" in
gpu_bench20)
(
# The driver's bench command (--steps 20 --warmup 5), repeated: headline spread.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/b20_rep.txt
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/b20_$i.json 2> gpurun_out/b20_$i.err || { tail gpurun_out/b20_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/b20_$i.json'));print('value',d['value'],'ms',d['ms_per_step'],'ungated',d.get('ungated_value'),d.get('ungated_ms_per_step'),'kernel_us',d['roofline']['kernel_us_avg'],'read_frac',d['roofline'].get('read_frac'))" >> gpurun_out/b20_rep.txt
done
cat gpurun_out/b20_rep.txt
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b20.json 2> gpurun_out/b20.err || { tail gpurun_out/b20.err; exit 1; }
cat gpurun_out/b20.json
)
;;
gpu_grid_ab)
(
# Config-3 grid balance A/B: workgroup width / resident
# workgroups per CU for the persistent batch kernel, timed by bench.py, plus the
# per-wave phase stamps of the diagnostic builds (loop end per wave) on tile8192.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
VARIANTS="default w8g2 w4 w7 w6" WLS="tile8192 tile8192_random batch" STEPS=256 \
  timeout -k 10 900 bash scripts/gpu_ab.sh > gpurun_out/grid_ab.txt 2>&1 || { cat gpurun_out/grid_ab.txt; exit 1; }
cat gpurun_out/grid_ab.txt
for v in w8 w8g2 w4; do
  echo "== stamps $v (tile8192)"
  MH_LIB=$GRAFT_REPO_ROOT/ab/lib_diag_$v.so timeout -k 10 120 python scripts/diag_stamps.py --tile8192 --tag _$v || exit 1
done
)
;;
gpu_kernarg_ab)
(
# HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device memory) vs the runtime default, interleaved
# on one box: driver-shaped frame bench and the long launches (eager and graph) -> gpurun_out/kernarg_ab.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/kernarg_ab.txt
run() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline $BARGS > gpurun_out/ka.json 2> gpurun_out/ka_err.txt || { tail gpurun_out/ka_err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ka.json')); r=d['roofline']; print('$tag', d['config']['workload'][:8], d['value'], 'kernel_us', r['kernel_us_avg'], d['config']['launch'][:30])" >> gpurun_out/kernarg_ab.txt
}
for rep in 1 2; do
  for ka in default 1; do
    E=(); [ $ka = 1 ] && E=(HIP_FORCE_DEV_KERNARG=1)
    BARGS="--steps 20 --warmup 5" run "rep$rep ka=$ka frame" "${E[@]}" X=1 || exit 1
    BARGS="--workload batch --steps 256 --warmup 256" run "rep$rep ka=$ka batch-eager" "${E[@]}" MH_BENCH_LONG=eager || exit 1
    BARGS="--workload batch --steps 256 --warmup 256" run "rep$rep ka=$ka batch-graph" "${E[@]}" MH_BENCH_LONG=graph || exit 1
  done
done
cat gpurun_out/kernarg_ab.txt
)
;;
gpu_long_ab2)
(
# Why are plain eager launches of the 64-frame batch slower than a graph replay? eager vs
# eager without the barrier bit (MH_BENCH_DIAG_RELAX=1) vs graph behind the gate, one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/long_ab2.txt
for rep in 1 2; do
  for mode in eager relax graph; do
    E=(MH_BENCH_LONG=eager); [ $mode = relax ] && E=(MH_BENCH_LONG=eager MH_BENCH_DIAG_RELAX=1); [ $mode = graph ] && E=(MH_BENCH_LONG=graph)
    env "${E[@]}" timeout -k 10 300 python bench.py --workload batch --steps 256 --warmup 256 --no-extras --no-cpu-baseline > gpurun_out/l2.json 2> gpurun_out/l2_err.txt || { tail gpurun_out/l2_err.txt; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/l2.json')); r=d['roofline']; print('rep $rep $mode', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', r['kernel_us_avg'], 'eager_med', r.get('eager_launch_us_median'))" >> gpurun_out/long_ab2.txt
  done
done
cat gpurun_out/long_ab2.txt
)
;;
gpu_long_ab)
(
# Long launches (64-frame batch, 8192^2 frame): plain eager region vs a hipGraph behind the
# launch gate (MH_BENCH_LONG=graph), interleaved on one box -> gpurun_out/long_ab.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/long_ab.txt
for rep in 1 2 3; do
  for mode in eager graph graph_ungated; do
    for wl in batch tile8192; do
      k=256; [ $wl = tile8192 ] && k=512
      MH_BENCH_LONG=$mode timeout -k 10 300 python bench.py --workload $wl --steps $k --warmup $k --no-extras --no-cpu-baseline > gpurun_out/long_$mode_$wl.json 2> gpurun_out/long_err.txt || { tail gpurun_out/long_err.txt; exit 1; }
      python3 -c "import json,sys; d=json.load(open('gpurun_out/long_$mode_$wl.json')); r=d['roofline']; print('rep $rep $mode $wl', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', r['kernel_us_avg'], 'frac', r['frac'], d['config']['launch'])" >> gpurun_out/long_ab.txt
    done
  done
done
cat gpurun_out/long_ab.txt
)
;;
gpu_r04_ab2)
(
# Round 4 A/B: the batch prologue's fixed table loads (default) vs the previous head; stamps
# of the new prologue on the cold 8192^2 tile; PMC of the batched encoder's kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r04_ab2.txt
: > $OUT
for rep in 1 2; do
  for v in default head; do
    if [ $v = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    for spec in batch:64:16 tile8192:64:16 tile8192_random:64:16 frame:20:5; do
      IFS=: read wl k w <<< "$spec"
      r=$(timeout -k 10 300 python bench.py --workload $wl --steps $k --warmup $w --no-extras --no-cpu-baseline 2>>gpurun_out/r04_ab2.err) || { echo "$v $wl FAILED" >> $OUT; exit 1; }
      echo "$v $wl $r" | python3 -c "import sys,json; l=sys.stdin.read().split(' ',2); d=json.loads(l[2]); print(l[0], l[1], 'value', d['value'], 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'])" >> $OUT
    done
  done
done
export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_stamps2.so
{ echo "== stamps --tile8192 --cold (fixed table loads)"; timeout -k 10 180 python3 scripts/diag_stamps.py --tile8192 --cold 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
unset MH_LIB
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"; do
  i=$((i+1)); rm -rf gpurun_out/pmc_enc/pmc$i
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_enc/pmc$i -o run -- python3 scripts/enc_batch_profile.py 64 2 > gpurun_out/pmc_enc$i.log 2>&1 || { tail gpurun_out/pmc_enc$i.log; exit 1; }
done
for k in enc_split_kernel enc_tree_batch_kernel enc_pack_batch_kernel; do
  { echo "== PMC $k (per dispatch)"; python3 scripts/pmc_summary.py gpurun_out/pmc_enc $k 1; } >> $OUT
done
cat $OUT
)
;;
gpu_r04_ab3)
(
# Round 4 A/B 3: batch prologue with the table loaded first and an LDS-only barrier (default)
# vs the round's head; stamps of the cold 8192^2 tile; the batched encoder's tests and trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_enc_batch.sh || exit 1
OUT=gpurun_out/r04_ab3.txt
: > $OUT
for rep in 1 2; do
  for v in default head; do
    if [ $v = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    for spec in batch:64:16 tile8192:64:16 tile8192_random:64:16; do
      IFS=: read wl k w <<< "$spec"
      r=$(timeout -k 10 300 python bench.py --workload $wl --steps $k --warmup $w --no-extras --no-cpu-baseline 2>>gpurun_out/r04_ab3.err) || { echo "$v $wl FAILED" >> $OUT; exit 1; }
      echo "$v $wl $r" | python3 -c "import sys,json; l=sys.stdin.read().split(' ',2); d=json.loads(l[2]); print(l[0], l[1], 'value', d['value'], 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'])" >> $OUT
    done
  done
done
export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_stamps2.so
{ echo "== stamps --tile8192 --cold (table first, LDS-only barrier)"; timeout -k 10 180 python3 scripts/diag_stamps.py --tile8192 --cold 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
unset MH_LIB
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_dec.log 2>&1 || { tail -30 gpurun_out/pytest_dec.log; exit 1; }
tail -1 gpurun_out/pytest_dec.log >> $OUT
cat $OUT
)
;;
gpu_r04_ab4)
(
# Round 4 A/B 4: the single-frame kernel's table barrier as an LDS-only barrier (default) vs
# __syncthreads (head: its fence waits for the span loads too). bench.py --workload frame
# (cold regions), interleaved three times, then the decode GPU tests on the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r04_ab4.txt
: > $OUT
for rep in 1 2 3; do
  for v in default head; do
    if [ $v = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    for spec in frame:20:5 frame:200:20; do
      IFS=: read wl k w <<< "$spec"
      r=$(timeout -k 10 300 python bench.py --workload $wl --steps $k --warmup $w --no-extras --no-cpu-baseline 2>>gpurun_out/r04_ab4.err) || { echo "$v $wl FAILED" >> $OUT; exit 1; }
      echo "$v $wl:$k $r" | python3 -c "import sys,json; l=sys.stdin.read().split(' ',2); d=json.loads(l[2]); print(l[0], l[1], 'value', d['value'], 'warm', d.get('warm_value'), 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'])" >> $OUT
    done
  done
done
unset MH_LIB
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_dec.log 2>&1 || { tail -30 gpurun_out/pytest_dec.log; exit 1; }
tail -1 gpurun_out/pytest_dec.log >> $OUT
cat $OUT
)
;;
gpu_r04_check)
(
# Round-4 GPU check: a full rebuild on the box, parity tests, smoke, the driver's bench command, a rocprofv3 kernel
# trace of the headline workload, the batched encoder and the multi-GPU C host (fail-fast).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
# the library the tests load is compiled and linked HERE, on the box,
# from this snapshot's sources (--force: every object and the link), not the pushed one
sha256sum metalhuffman_amd/libmetalhuffman_amd.so > gpurun_out/build_on_box.log
timeout -k 10 900 python -m metalhuffman_amd.build --force >> gpurun_out/build_on_box.log 2>&1 || { tail -20 gpurun_out/build_on_box.log; exit 1; }
sha256sum metalhuffman_amd/libmetalhuffman_amd.so >> gpurun_out/build_on_box.log
grep -c -- "--offload-arch=gfx950" gpurun_out/build_on_box.log; tail -1 gpurun_out/build_on_box.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log; grep -c PASSED gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log | tail -1
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
rm -rf gpurun_out/prof_frame
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_frame -o run -- python3 bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/bench_prof_frame.json 2> gpurun_out/bench_prof_frame.err || { tail gpurun_out/bench_prof_frame.err; exit 1; }
{ echo "== bench.py --workload frame --steps 20 --warmup 5 (profiled line: roofline.kernel_us_avg $(python3 -c "import json;print(json.load(open('gpurun_out/bench_prof_frame.json'))['roofline']['kernel_us_avg'])"))"; python3 scripts/ktrace_summary.py gpurun_out/prof_frame 20 1; } > gpurun_out/ktrace_summary.txt
cat gpurun_out/ktrace_summary.txt
rm -rf gpurun_out/prof_encb
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_encb -o run -- python3 scripts/enc_batch_profile.py 64 8 > gpurun_out/enc_batch.log 2>&1 || { tail gpurun_out/enc_batch.log; exit 1; }
cat gpurun_out/enc_batch.log | grep batch
python3 - <<'PY'
import csv
for r in sorted(csv.DictReader(open("gpurun_out/prof_encb/run_kernel_stats.csv")), key=lambda r: -float(r["TotalDurationNs"]))[:6]:
    print(f"{float(r['AverageNs']) / 1e3:9.2f} us  x{r['Calls']:>4}  {r['Name'][:90]}")
PY
python3 -c "import numpy as np, sys; sys.path.insert(0,'.'); from metalhuffman_amd import frames as F; open('gpurun_out/bb.gray','wb').write(np.ascontiguousarray(F.bigbridge()).tobytes())"
timeout -k 10 120 ./host/mh_decode_multi 1 64 20 2048 1536 gpurun_out/bb.gray > gpurun_out/multi.log 2>&1 || { cat gpurun_out/multi.log; exit 1; }
cat gpurun_out/multi.log
rm -f gpurun_out/bb.gray
)
;;
gpu_r04_frame_stamps)
(
# Cold and warm phase stamps of the single-frame launch (config 2) from a MH_DIAG_STAMPS=1 build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_stamps.so
OUT=gpurun_out/r04_frame_stamps.txt
{ echo "== stamps single frame --cold"; timeout -k 10 180 python3 scripts/diag_stamps.py --cold 2>&1 | grep -v amdgpu.ids; } > $OUT || exit 1
{ echo "== stamps single frame (warm)"; timeout -k 10 180 python3 scripts/diag_stamps.py 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
cat $OUT
)
;;
gpu_r04_kernarg_ab)
(
# Kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) vs the runtime default, on the
# single-frame workload (cold regions) and the stamped launch (entry -> first header).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r04_kernarg_ab.txt
: > $OUT
for rep in 1 2 3; do
  for v in default devkernarg; do
    if [ $v = devkernarg ]; then export HIP_FORCE_DEV_KERNARG=1; else unset HIP_FORCE_DEV_KERNARG; fi
    for spec in frame:20:5 batch:20:5; do
      IFS=: read wl k w <<< "$spec"
      r=$(timeout -k 10 300 python bench.py --workload $wl --steps $k --warmup $w --no-extras --no-cpu-baseline 2>>gpurun_out/r04_kernarg_ab.err) || { echo "$v $wl FAILED" >> $OUT; exit 1; }
      echo "$v $wl:$k $r" | python3 -c "import sys,json; l=sys.stdin.read().split(' ',2); d=json.loads(l[2]); print(l[0], l[1], 'value', d['value'], 'warm', d.get('warm_value'), 'ungated', d.get('ungated_value'), 'kernel_us', d['roofline']['kernel_us_avg'])" >> $OUT
    done
  done
done
export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_stamps.so
for v in default devkernarg; do
  if [ $v = devkernarg ]; then export HIP_FORCE_DEV_KERNARG=1; else unset HIP_FORCE_DEV_KERNARG; fi
  { echo "== stamps single frame (warm) $v"; timeout -k 10 180 python3 scripts/diag_stamps.py 2>&1 | grep -v amdgpu.ids | grep -E "entry|hdr|launch|decomposition"; } >> $OUT || exit 1
done
cat $OUT
)
;;
gpu_r04_tile_ab)
(
# Round 4: (1) VMEM-refill A/B on the batch kernel: bench + one PMC pass
# each; (2) per-wave phase stamps of the 8192^2 tile and the 64-frame batch, cold and warm
# (start / steady / drain).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r04_ab.txt
: > $OUT
for rep in 1 2; do
  for v in default vmemrefill; do
    if [ $v = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    for wl in batch tile8192; do
      r=$(timeout -k 10 300 python bench.py --workload $wl --steps 64 --warmup 16 --no-extras --no-cpu-baseline 2>>gpurun_out/r04_ab.err) || { echo "$v $wl FAILED" >> $OUT; exit 1; }
      echo "$v $wl $r" | python3 -c "import sys,json; l=sys.stdin.read().split(' ',2); d=json.loads(l[2]); print(l[0], l[1], 'value', d['value'], 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'])" >> $OUT
    done
  done
done
for v in default vmemrefill; do
  if [ $v = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
  rm -rf gpurun_out/pmc_$v; mkdir -p gpurun_out/pmc_$v
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_$v/pmc1 -o run -- python3 bench.py --workload batch --steps 16 --warmup 2 --no-extras --no-cpu-baseline > gpurun_out/pmc_$v.log 2>&1 || { tail gpurun_out/pmc_$v.log; exit 1; }
  { echo "== PMC $v batch (mh_decode_kernel, per dispatch)"; python3 scripts/pmc_summary.py gpurun_out/pmc_$v mh_decode_kernel 2; } >> $OUT
done
unset MH_LIB
export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_stamps.so
for args in "--tile8192 --cold" "--tile8192" "--batch 64 --cold"; do
  { echo "== stamps $args"; timeout -k 10 180 python3 scripts/diag_stamps.py $args 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
done
cat $OUT
)
;;
gpu_window_ab)
(
# Long-launch timed region A/B: all K/16 graph replays queued behind the launch gate
# (MH_BENCH_LONG=graph) vs only the first (window, the default), unprofiled and under
# rocprofv3 --kernel-trace (timed_steady from the trace markers).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/window_ab.txt
: > $OUT
for rep in 1 2; do
  for m in graph window; do
    for wl in batch tile8192; do
      r=$(MH_BENCH_LONG=$m timeout -k 10 300 python bench.py --workload $wl --steps 256 --warmup 64 --no-extras --no-cpu-baseline 2>>gpurun_out/window_ab.err) || exit 1
      echo "$r" | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$m $wl value', d['value'], 'kernel_us', r['kernel_us_avg'], 'region_us', r['region_us_per_launch'], 'graph_us', r['graph_us_per_launch'])" >> $OUT
    done
  done
done
for m in graph window; do
  for wl in batch tile8192; do
    rm -rf gpurun_out/wprof_${m}_$wl
    MH_BENCH_LONG=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wprof_${m}_$wl -o run -- \
      python3 bench.py --workload $wl --steps 256 --warmup 64 --no-extras --no-cpu-baseline > gpurun_out/wprof_${m}_$wl.json 2>gpurun_out/wprof.err || exit 1
    k=$(python3 -c "import json; print(json.loads(open('gpurun_out/wprof_${m}_$wl.json').read().strip().splitlines()[-1])['roofline']['kernel_us_avg'])")
    echo "== profiled $m $wl: line kernel_us_avg $k" >> $OUT
    python3 scripts/ktrace_summary.py gpurun_out/wprof_${m}_$wl 256 16 >> $OUT || exit 1
  done
done
cat $OUT
)
;;
*) echo "unknown session $1"; exit 2 ;;
esac

# Round 5's GPU sessions (folded in round 6)
# Each former one-off GPU session script is one case below, verbatim (the profiles/ record each produced
# is named in its header comment). Run one as:  bash scripts/gpu_r05_sessions.sh <name>
# names: gpu_r05_bisect gpu_r05_final2 gpu_r05_session1 gpu_r05_session2 gpu_r05_session3 gpu_r05_session4 gpu_r05_session5 gpu_r05_session6 gpu_r05_session9 gpu_r05_session11 gpu_r05_session12 gpu_r05_session13 gpu_r05_session14 gpu_r05_session15 gpu_r05_session16 gpu_r05_session17 gpu_r05_session18 gpu_r05_session19 gpu_r05_session20 gpu_r05_session21 gpu_r05_session22 gpu_r05_session23 gpu_r05_session24 gpu_r05_session25 gpu_r05_session26 gpu_r05_session27 gpu_r05_session28 gpu_r05_session29 gpu_r05_session30 gpu_r05_session31
set -o pipefail
case "$1" in
gpu_r05_bisect)
(
# Round 5: bisect of the round-4 batch-kernel regression on ONE box,
# interleaved: r03 head (f433465), 8397e6d (single flavour-switched loop + kernel args),
# HEAD r04 (7dc48b7 prologue), and "split" (the r05 tree: r04 prologue + one loop
# instantiation per flavour); workloads batch / tile8192 / tile8192_random; then one
# PMC pass per variant on the batch.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_bisect.txt
: > $OUT
VARS=${VARS:-"r03 c8397 head split"}
for rep in 1 2; do
  for v in $VARS; do
    if [ $v = split ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    for wl in ${WLS:-batch tile8192 tile8192_random}; do
      r=$(timeout -k 10 150 python bench.py --workload $wl --steps 64 --warmup 16 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_bisect.err) || { echo "$v $wl FAILED" >> $OUT; exit 1; }
      echo "$v $wl $r" | python3 -c "import sys,json; l=sys.stdin.read().split(' ',2); d=json.loads(l[2]); print(l[0], l[1], 'value', d['value'], 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'])" >> $OUT
      echo "rep $rep $v $wl done"
    done
  done
done
if [ -n "$PMC" ]; then
for v in $VARS; do
  if [ $v = split ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
  rm -rf gpurun_out/pmc_$v; mkdir -p gpurun_out/pmc_$v
  timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_$v/pmc1 -o run -- python3 bench.py --workload batch --steps 16 --warmup 2 --no-extras --no-cpu-baseline > gpurun_out/pmc_$v.log 2>&1 || { tail gpurun_out/pmc_$v.log; exit 1; }
  { echo "== PMC $v batch (mh_decode_kernel, per dispatch)"; python3 scripts/pmc_summary.py gpurun_out/pmc_$v mh_decode_kernel 2; } >> $OUT
  echo "pmc $v done"
done
fi
cat $OUT
)
;;
gpu_r05_final2)
(
# Round 5, last GPU call: the final check at HEAD (scripts/gpu_r05_check.sh: build --force on
# the box, the whole GPU suite, smoke, the driver's bench command, rocprofv3 traces, encoders,
# plain-C multi host), then session 24's A/B of the single-frame flat 8-bit path:
# uniform-random 2048x1536 one-frame launches (time_frame.py --random) and the config-2 frame
# command as a control, default vs noflat8 (MH_FLAT8=0), interleaved x 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_r05_check.sh > gpurun_out/r05_check3.txt 2>&1 || { tail -40 gpurun_out/r05_check3.txt; exit 1; }
echo "check done"
OUT=gpurun_out/r05_flat8_small_ab.txt
: > $OUT
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'])"; }
for rep in 1 2 3; do
  for v in default noflat8; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    timeout -k 10 120 python3 scripts/time_frame.py --random --tag $v 2>>gpurun_out/r05_flat8_small_ab.err | tail -1 >> $OUT || { echo "$v FAILED" >> $OUT; exit 1; }
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_flat8_small_ab.err) || { echo "$v frame FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
tail -30 gpurun_out/r05_check3.txt
cat $OUT
)
;;
gpu_r05_session1)
(
# Round 5, GPU session 1: the whole GPU suite on this tree (split batch loop, lane pairs
# in the diagnostic library, fork-safe CPU pool, encoder tile tails, rank devices), then
# the batch-kernel bisect (scripts/gpu_r05_bisect.sh, no PMC).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r05_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r05_pytest_gpu.log
bash scripts/gpu_r05_bisect.sh
)
;;
gpu_r05_session2)
(
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
)
;;
gpu_r05_session3)
(
# Round 5, GPU session 3: the whole GPU suite on this tree; the batched encoder A/B
# (default = this tree: tile tails kept by the split; encr04 = round-4 encoder; enc256 =
# tile tails + 256-block batch tiles) with HIP-event timing and HBM traffic per variant;
# rocprofv3 kernel traces of batch / tile8192 / tile8192_random at this HEAD (VERDICT r04
# item 2).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r05_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r05_pytest_gpu.log
OUT=gpurun_out/r05_enc_ab.txt
: > $OUT
VARIANTS="encr04 enc256"
for rep in 1 2 3; do
  for v in default $VARIANTS; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    timeout -k 10 120 python3 scripts/enc_batch_profile.py 64 8 2>&1 | grep "^batch" | tail -1 | sed "s/^/$v /" >> $OUT || exit 1
  done
done
echo "enc timing done"
for v in default $VARIANTS; do
  if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
  for ctr in FETCH_SIZE WRITE_SIZE; do
    d=gpurun_out/pmc_enc_${v}_$ctr
    rm -rf $d
    timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $GRAFT_REPO_ROOT/$d/pmc -o run -- python3 scripts/enc_batch_profile.py 64 2 > $d.log 2>&1 || { echo "pmc $v $ctr failed"; tail -5 $d.log; exit 1; }
  done
  alg=$(grep -o "alg_bytes [0-9]*" gpurun_out/pmc_enc_${v}_FETCH_SIZE.log | head -1 | cut -d" " -f2)
  { echo "== traffic $v"; python3 scripts/enc_batch_pmc.py gpurun_out/pmc_enc_${v}_FETCH_SIZE gpurun_out/pmc_enc_${v}_WRITE_SIZE --alg $alg; } >> $OUT 2>&1
  echo "traffic $v done"
done
unset MH_LIB
cat $OUT
: > gpurun_out/r05_ktrace_summary.txt
for spec in frame:20:5 batch:256:256 tile8192:512:512 tile8192_random:512:512; do
  IFS=: read wl k w <<< "$spec"
  rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_$wl
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$wl -o run -- python3 bench.py --workload $wl --steps $k --warmup $w --no-extras --no-cpu-baseline > gpurun_out/bench_prof_$wl.json 2> gpurun_out/bench_prof_$wl.err || { tail gpurun_out/bench_prof_$wl.err; exit 1; }
  u=$(python3 -c "import json;print(json.load(open('gpurun_out/bench_prof_$wl.json'))['roofline'].get('kernel_us_steady_unit') or 1)")
  { echo "== bench.py --workload $wl --steps $k --warmup $w (profiled line: roofline.kernel_us_avg $(python3 -c "import json;print(json.load(open('gpurun_out/bench_prof_$wl.json'))['roofline']['kernel_us_avg'])"), steady unit $u)"; python3 scripts/ktrace_summary.py gpurun_out/prof_$wl $k $u; } >> gpurun_out/r05_ktrace_summary.txt
  echo "ktrace $wl done"
done
cat gpurun_out/r05_ktrace_summary.txt
)
;;
gpu_r05_session4)
(
# Round 5, GPU session 4: batched encoder at 256-block tiles (default) vs 128 / 512:
# encoder GPU tests, HIP-event timing (3 reps interleaved), a kernel trace per variant
# (per-kernel split), HBM traffic of enc512.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode_batch.py tests/test_gpu_encode.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05_pytest_enc.log 2>&1 || { tail -40 gpurun_out/r05_pytest_enc.log; exit 1; }
tail -1 gpurun_out/r05_pytest_enc.log
OUT=gpurun_out/r05_enc_ab2.txt
: > $OUT
VARIANTS="enc128 enc512"
for rep in 1 2 3; do
  for v in default $VARIANTS; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    timeout -k 10 120 python3 scripts/enc_batch_profile.py 64 8 2>&1 | grep "^batch" | tail -1 | sed "s/^/$v /" >> $OUT || exit 1
  done
done
for v in default $VARIANTS; do
  if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
  rm -rf gpurun_out/prof_ab_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_ab_$v -o run -- python3 scripts/enc_batch_profile.py 64 8 > gpurun_out/prof_ab_$v.log 2>&1 || { tail gpurun_out/prof_ab_$v.log; exit 1; }
  python3 - "$v" <<'PY' >> $OUT
import csv, sys
v = sys.argv[1]
for r in sorted(csv.DictReader(open(f"gpurun_out/prof_ab_{v}/run_kernel_stats.csv")), key=lambda r: -float(r["TotalDurationNs"]))[:3]:
    print(f"{v} kernel {float(r['AverageNs']) / 1e3:9.2f} us  x{r['Calls']:>4}  {r['Name'][:70]}")
PY
done
for v in enc512; do
  export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so
  for ctr in FETCH_SIZE WRITE_SIZE; do
    d=gpurun_out/pmc_enc_${v}_$ctr
    rm -rf $d
    timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $GRAFT_REPO_ROOT/$d/pmc -o run -- python3 scripts/enc_batch_profile.py 64 2 > $d.log 2>&1 || { echo "pmc $v $ctr failed"; tail -5 $d.log; exit 1; }
  done
  alg=$(grep -o "alg_bytes [0-9]*" gpurun_out/pmc_enc_${v}_FETCH_SIZE.log | head -1 | cut -d" " -f2)
  { echo "== traffic $v"; python3 scripts/enc_batch_pmc.py gpurun_out/pmc_enc_${v}_FETCH_SIZE gpurun_out/pmc_enc_${v}_WRITE_SIZE --alg $alg; } >> $OUT 2>&1
done
unset MH_LIB
cat $OUT
)
;;
gpu_r05_session5)
(
# Round 5, GPU session 5: H2D probe (config 5: is one copy stream the limit?), the 2-rank
# gloo rehearsal of the N > 1 bench path (rank_devices at world 2), and a randomized parity
# sweep at this HEAD (decode paths + single-frame and batched GPU encode).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python3 scripts/h2d_probe.py > gpurun_out/r05_h2d_probe.txt 2>&1 || { cat gpurun_out/r05_h2d_probe.txt; exit 1; }
cat gpurun_out/r05_h2d_probe.txt
bash scripts/gpu_rehearse_n2.sh > gpurun_out/r05_rehearse_n2.txt 2>&1 || { cat gpurun_out/r05_rehearse_n2.txt; exit 1; }
cat gpurun_out/r05_rehearse_n2.txt
MH_STRESS_SECONDS=300 MH_STRESS_FIRST_CASE=120000 bash scripts/gpu_stress_long.sh
cp gpurun_out/stress_long.log gpurun_out/r05_stress.log
)
;;
gpu_r05_session6)
(
# Round 5, GPU session 6: does the cold-region flush itself slow the first launch of a
# region? bench.py's flush is a 512 MiB device copy (dirty lines left behind); A/B against
# a read-only eviction (MH_BENCH_FLUSH=read: a reduction over 1 GiB, nothing dirty), on
# the driver's frame command and the batch / tile workloads, interleaved; then per-wave
# stamps of the first launch after each kind of flush.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_flush_ab.txt
: > $OUT
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'warm', d.get('warm_value'))"; }
for rep in 1 2 3; do
  for mode in copy read; do
    for spec in frame:20:5 batch:64:16 tile8192:64:16; do
      IFS=: read wl k w <<< "$spec"
      r=$(MH_BENCH_FLUSH=$mode timeout -k 10 150 python bench.py --workload $wl --steps $k --warmup $w --no-extras --no-cpu-baseline 2>>gpurun_out/r05_flush_ab.err) || { echo "$mode $wl FAILED" >> $OUT; exit 1; }
      echo "$mode $wl $(echo "$r" | line)" >> $OUT
    done
  done
  echo "rep $rep done"
done
export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_stamps.so
for mode in copy read; do
  { echo "== stamps single frame --cold, flush $mode"; MH_BENCH_FLUSH=$mode timeout -k 10 180 python3 scripts/diag_stamps.py --cold 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
done
cat $OUT
)
;;
gpu_r05_session9)
(
# Round 5, GPU session 9: tiled split without dead per-row stores (encoder GPU tests, then
# default vs encprev = the encoder before this change, 3 reps interleaved + per-kernel trace).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode_batch.py tests/test_gpu_encode.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05_pytest_enc2.log 2>&1 || { tail -40 gpurun_out/r05_pytest_enc2.log; exit 1; }
tail -1 gpurun_out/r05_pytest_enc2.log
OUT=gpurun_out/r05_enc_ab3.txt
: > $OUT
VARIANTS="encprev"
for rep in 1 2 3; do
  for v in default $VARIANTS; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    timeout -k 10 120 python3 scripts/enc_batch_profile.py 64 8 2>&1 | grep "^batch" | tail -1 | sed "s/^/$v /" >> $OUT || exit 1
  done
done
for v in default $VARIANTS; do
  if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
  rm -rf gpurun_out/prof_ab_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_ab_$v -o run -- python3 scripts/enc_batch_profile.py 64 8 > gpurun_out/prof_ab_$v.log 2>&1 || { tail gpurun_out/prof_ab_$v.log; exit 1; }
  python3 - "$v" <<'PY' >> $OUT
import csv, sys
v = sys.argv[1]
for r in sorted(csv.DictReader(open(f"gpurun_out/prof_ab_{v}/run_kernel_stats.csv")), key=lambda r: -float(r["TotalDurationNs"]))[:3]:
    print(f"{v} kernel {float(r['AverageNs']) / 1e3:9.2f} us  x{r['Calls']:>4}  {r['Name'][:70]}")
PY
done
unset MH_LIB
cat $OUT
)
;;
gpu_r05_session11)
(
# Round 5, GPU session 11: kernarg preload for the decode kernels (the leading scalar
# arguments in SGPRs at wave launch): decode GPU tests, then default vs decprev (the
# kernels taking only the DecodeArgs struct: nothing preloaded), interleaved: the driver's
# frame command (20 steps) x 4, batch and 8192^2 x 2.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_lane_pairs.py tests/test_check.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05_pytest_dec.log 2>&1 || { tail -40 gpurun_out/r05_pytest_dec.log; exit 1; }
tail -1 gpurun_out/r05_pytest_dec.log
OUT=gpurun_out/r05_preload_ab.txt
: > $OUT
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'warm', d.get('warm_value'), 'ungated', d.get('ungated_value'))"; }
for rep in 1 2 3 4; do
  for v in default decprev; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    specs="frame:20:5"
    if [ $rep -le 2 ]; then specs="frame:20:5 batch:64:16 tile8192:64:16"; fi
    for spec in $specs; do
      IFS=: read wl k w <<< "$spec"
      r=$(timeout -k 10 150 python bench.py --workload $wl --steps $k --warmup $w --no-extras --no-cpu-baseline 2>>gpurun_out/r05_preload_ab.err) || { echo "$v $wl FAILED" >> $OUT; exit 1; }
      echo "$v $wl $(echo "$r" | line)" >> $OUT
    done
  done
  echo "rep $rep done"
done
unset MH_LIB
cat $OUT
)
;;
gpu_r05_session12)
(
# Round 5, GPU session 12: the single-frame kernel's workgroup width again after the kernarg
# preload (4 waves = one per SIMD, default; 8 = two per SIMD, half the workgroups; 2), on the
# driver's frame command, interleaved x 3; then per-wave stamps of the current kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_small_wg_ab.txt
: > $OUT
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'warm', d.get('warm_value'))"; }
for rep in 1 2 3; do
  for v in default small8 small2; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_small_wg_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_stamps.so
{ echo "== stamps single frame --cold"; timeout -k 10 180 python3 scripts/diag_stamps.py --cold 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
{ echo "== stamps single frame (warm)"; timeout -k 10 180 python3 scripts/diag_stamps.py 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
cat $OUT
)
;;
gpu_r05_session13)
(
# Round 5, GPU session 13: the single-frame kernel's row-store cache policy under the cold
# method (round 3 chose write-through nt sc1 on warm regions): default (nt sc1 = 18) vs nt
# (2) vs default policy (0) vs sc1 (16); driver frame command, interleaved x 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_small_store_ab.txt
: > $OUT
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'warm', d.get('warm_value'))"; }
for rep in 1 2 3 4; do
  for v in default st_nt st_def st_sc1; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_small_store_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
cat $OUT
)
;;
gpu_r05_session14)
(
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
)
;;
gpu_r05_session15)
(
# Round 5, GPU session 15: the single-frame kernel with its 8-row loop rolled (1,203 instead
# of 4,751 instructions: every launch refetches its code after the dispatch's cache
# invalidation) vs the unrolled default; decode tests with the variant, then the driver's
# frame command interleaved x 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
MH_LIB=$GRAFT_REPO_ROOT/ab/lib_rolled.so timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05_pytest_rolled.log 2>&1 || { tail -40 gpurun_out/r05_pytest_rolled.log; exit 1; }
tail -1 gpurun_out/r05_pytest_rolled.log
OUT=gpurun_out/r05_rolled_ab.txt
: > $OUT
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'warm', d.get('warm_value'))"; }
for rep in 1 2 3 4; do
  for v in default rolled; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_rolled_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
done
cat $OUT
)
;;
gpu_r05_session16)
(
# Round 5, GPU session 16: the single-frame kernel with its eight row stores issued after the
# whole block (8 x 2 registers held) instead of after each row, so no store issues between
# the steps of the chain (cold, the chain ran 3.16 us vs 2.68 us warm); decode tests with
# the variant, then the driver's frame command interleaved x 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
MH_LIB=$GRAFT_REPO_ROOT/ab/lib_defer.so timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05_pytest_defer.log 2>&1 || { tail -40 gpurun_out/r05_pytest_defer.log; exit 1; }
tail -1 gpurun_out/r05_pytest_defer.log
OUT=gpurun_out/r05_defer_ab.txt
: > $OUT
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'warm', d.get('warm_value'))"; }
for rep in 1 2 3 4; do
  for v in default defer; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_defer_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
done
cat $OUT
)
;;
gpu_r05_session17)
(
# Round 5, GPU session 17: why the single-frame decode chain runs ~0.45 us longer cold than warm.
# Stamps with core-clock cycles (MH_DIAG_CLOCK), the same with every row store dropped, and with
# an entry-time touch of the tile's output rows and codes page (MH_SMALL_TOUCH); then the driver's
# frame command, default vs touch vs lazy refill (MH_SMALL_LAZY), interleaved x 3, after the
# lazy variant's decode parity tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_chain_cold_ab.txt
: > $OUT
echo "== pytest decode, lazy refill" >> $OUT
MH_LIB=$GRAFT_REPO_ROOT/ab/lib_lazy.so timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_stress.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_lazy.log 2>&1
rc=$?
tail -3 gpurun_out/r05_pytest_lazy.log >> $OUT
echo "pytest rc $rc" >> $OUT
# a wrong-output failure (1) is a result; a fault, abort or time limit ends the call
[ $rc -le 1 ] || exit 1
LAZY_OK=$rc
for v in stampclk stampclk_nostore stampclk_touch stampclk_lazy; do
  export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so
  { echo "== $v --cold"; timeout -k 10 180 python3 scripts/diag_stamps.py --cold --clock --tag _$v 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
  { echo "== $v warm"; timeout -k 10 180 python3 scripts/diag_stamps.py --clock --tag _$v 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
  echo "$v stamps done"
done
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'warm', d.get('warm_value'))"; }
for rep in 1 2 3; do
  for v in default touch lazy; do
    [ "$v" = lazy ] && [ "$LAZY_OK" != 0 ] && continue
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_chain_cold_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
cat $OUT
)
;;
gpu_r05_session18)
(
# Round 5, GPU session 18: the lazy-refill step (MH_SMALL_LAZY=1, ab/lib_lazy.so) -- every GPU
# test through it, then the driver's frame command default vs lazy, interleaved x 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_lazy_ab.txt
: > $OUT
echo "== pytest -m gpu, lazy refill library" >> $OUT
MH_LIB=$GRAFT_REPO_ROOT/ab/lib_lazy.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_lazy.log 2>&1 || { tail -5 gpurun_out/r05_pytest_lazy.log >> $OUT; exit 1; }
tail -2 gpurun_out/r05_pytest_lazy.log >> $OUT
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'warm', d.get('warm_value'))"; }
for rep in 1 2 3 4; do
  for v in default lazy; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_lazy_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
cat $OUT
)
;;
gpu_r05_session19)
(
# Round 5, GPU session 19: lazy refill now the default. A codes-page touch at entry
# (MH_SMALL_TOUCH=2: one load per wave at the tile's linear share of the codes, in flight with
# the block offsets) -- stamps cold, then the driver's frame command default vs touch2 vs the
# old eager refill (nolazy), interleaved x 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_touch2_ab.txt
: > $OUT
for v in stampclk stampclk_touch2; do
  export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so
  { echo "== $v --cold"; timeout -k 10 180 python3 scripts/diag_stamps.py --cold --clock --tag _$v 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
  echo "$v stamps done"
done
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'warm', d.get('warm_value'))"; }
for rep in 1 2 3; do
  for v in default touch2 nolazy; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_touch2_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
cat $OUT
)
;;
gpu_r05_session20)
(
# Round 5, GPU session 20: the batch kernel with the single-level 14-bit table for tables whose
# longest code is 14 bits (MH_BATCH_L14=1, ab/lib_bl14.so: no escape test, 2 workgroups per CU
# by LDS instead of 3). Decode GPU tests through it, then batch / tile8192 / tile8192_random,
# default vs bl14, interleaved x 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_batch_l14_ab.txt
: > $OUT
echo "== pytest decode + stress, bl14 library" >> $OUT
MH_LIB=$GRAFT_REPO_ROOT/ab/lib_bl14.so timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_stress.py tests/test_check.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_bl14.log 2>&1
rc=$?
tail -3 gpurun_out/r05_pytest_bl14.log >> $OUT
[ $rc -le 1 ] || exit 1
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'])"; }
for rep in 1 2 3; do
  for wl in batch tile8192 tile8192_random; do
    for v in default bl14; do
      if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
      r=$(timeout -k 10 150 python bench.py --workload $wl --steps 64 --warmup 32 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_batch_l14_ab.err) || { echo "$v $wl FAILED" >> $OUT; exit 1; }
      echo "$v $wl $(echo "$r" | line)" >> $OUT
    done
  done
  echo "rep $rep done"
done
cat $OUT
)
;;
gpu_r05_session21)
(
# Round 5, GPU session 21: the lazy-refill default under new cases -- the refill-extreme GPU
# tests, then a 5-minute randomized parity sweep at this HEAD (new case ids from 200000).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -v -k "refill_extremes or small_launch or long_codes" --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_refill_extremes.log 2>&1 || { tail -30 gpurun_out/r05_pytest_refill_extremes.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r05_pytest_refill_extremes.log | tail -12
MH_STRESS_SECONDS=300 MH_STRESS_FIRST_CASE=200000 bash scripts/gpu_stress_long.sh
cp gpurun_out/stress_long.log gpurun_out/r05_stress_head2.log
tail -4 gpurun_out/r05_stress_head2.log
)
;;
gpu_r05_session22)
(
# Round 5, GPU session 22: the batch kernel's flat 8-bit path (byte arithmetic, no table
# lookups; MH_BATCH_FLAT8). The decode GPU tests (new flat8 formats included), then the
# uniform-random 8192^2 tile (config 3 stress) and the batch / 8192^2 BigBridge tile as a
# control, default vs noflat8 (the general flat step), interleaved x 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_flat8_ab.txt
: > $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_check.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_flat8.log 2>&1
rc=$?
tail -3 gpurun_out/r05_pytest_flat8.log >> $OUT
echo "pytest rc $rc" >> $OUT
[ $rc -eq 0 ] || { tail -40 gpurun_out/r05_pytest_flat8.log; exit 1; }
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'])"; }
for rep in 1 2 3; do
  for wl in tile8192_random batch; do
    for v in default noflat8; do
      if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
      r=$(timeout -k 10 150 python bench.py --workload $wl --steps 64 --warmup 32 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_flat8_ab.err) || { echo "$v $wl FAILED" >> $OUT; exit 1; }
      echo "$v $wl $(echo "$r" | line)" >> $OUT
    done
  done
  echo "rep $rep done"
done
cat $OUT
)
;;
gpu_r05_session23)
(
# Round 5, GPU session 23: flat 8-bit path variants on the uniform-random 8192^2 tile --
# default (per-lane loads, one tile of codes ahead), f8staged (batch_loop's coalesced span
# loads and LDS stage, byte arithmetic from the stage), f8prio (default + wave priority by
# tiles left), noflat8 (the general flat step); flat tests through f8staged first.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_flat8_variants_ab.txt
: > $OUT
MH_LIB=$GRAFT_REPO_ROOT/ab/lib_f8staged.so timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -q -k "flat" --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_f8staged.log 2>&1
rc=$?
tail -2 gpurun_out/r05_pytest_f8staged.log >> $OUT
[ $rc -le 1 ] || exit 1
STAGED_OK=$rc
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'])"; }
for rep in 1 2 3; do
  for v in default f8staged f8prio noflat8; do
    [ "$v" = f8staged ] && [ "$STAGED_OK" != 0 ] && continue
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload tile8192_random --steps 64 --warmup 32 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_flat8_variants_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v tile8192_random $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
cat $OUT
)
;;
gpu_r05_session24)
(
# Round 5, GPU session 24: flat 8-bit tables in the single-frame kernel too (byte arithmetic
# from the staged span). The whole GPU suite, then one-frame launches of uniform-random
# 2048x1536 frames (time_frame.py --random, graph of 200 launches) and the driver's config-2
# frame command as a control, default vs noflat8 (MH_FLAT8=0), interleaved x 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_flat8_small_ab.txt
: > $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05_pytest_flat8_all.log 2>&1 || { tail -30 gpurun_out/r05_pytest_flat8_all.log; exit 1; }
tail -1 gpurun_out/r05_pytest_flat8_all.log >> $OUT
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'])"; }
for rep in 1 2 3; do
  for v in default noflat8; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    timeout -k 10 120 python3 scripts/time_frame.py --random --tag $v 2>>gpurun_out/r05_flat8_small_ab.err | tail -1 >> $OUT || { echo "$v FAILED" >> $OUT; exit 1; }
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_flat8_small_ab.err) || { echo "$v frame FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
cat $OUT
)
;;
gpu_r05_session25)
(
# Round 5, GPU session 25: a 5-minute randomized parity sweep at the final HEAD (the flat 8-bit
# paths included: the sweep's "uniform" frames), new case ids from 300000.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
MH_STRESS_SECONDS=300 MH_STRESS_FIRST_CASE=300000 bash scripts/gpu_stress_long.sh
cp gpurun_out/stress_long.log gpurun_out/r05_stress_head3.log
tail -4 gpurun_out/r05_stress_head3.log
)
;;
gpu_r05_session26)
(
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
)
;;
gpu_r05_session27)
(
# Round 5, GPU session 27: the flat 8-bit batch path on the uniform-random 8192^2 tile (16,384
# tiles, 2.67 per wave): default (one tile of codes ahead), f8aux18 (write-through row stores),
# f8g2 (two tiles per round trip, flat8_loop_grouped), f8g2aux18; the flat tests through f8g2
# first; interleaved x 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_flat8_group_ab.txt
: > $OUT
MH_LIB=$GRAFT_REPO_ROOT/ab/lib_f8g2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -q -k "flat" --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_f8g2.log 2>&1
rc=$?
tail -2 gpurun_out/r05_pytest_f8g2.log >> $OUT
[ $rc -le 1 ] || exit 1
G_OK=$rc
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'], 'frac', d['roofline']['frac'])"; }
for rep in 1 2 3; do
  for v in default f8aux18 f8g2 f8g2aux18; do
    case $v in f8g2*) [ "$G_OK" != 0 ] && continue;; esac
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload tile8192_random --steps 64 --warmup 32 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_flat8_group_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v tile8192_random $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
cat $OUT
)
;;
gpu_r05_session28)
(
# Round 5, GPU session 28: an 8-minute randomized parity sweep at the final HEAD, new case ids
# from 400000.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
MH_STRESS_SECONDS=480 MH_STRESS_FIRST_CASE=400000 bash scripts/gpu_stress_long.sh
cp gpurun_out/stress_long.log gpurun_out/r05_stress_head4.log
tail -4 gpurun_out/r05_stress_head4.log
)
;;
gpu_r05_session29)
(
# Round 5, GPU session 29: the lazy step's next-word read as a broadcast for lanes that did not
# refill (MH_SMALL_LAZY_BCAST=1, ab/lib_lzbc.so: only refilling lanes' reads can conflict; the
# read's select deferred one step). Decode tests through it, then the driver's frame command,
# default vs lzbc, interleaved x 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_lazy_bcast_ab.txt
: > $OUT
MH_LIB=$GRAFT_REPO_ROOT/ab/lib_lzbc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_stress.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_lzbc.log 2>&1
rc=$?
tail -2 gpurun_out/r05_pytest_lzbc.log >> $OUT
[ $rc -le 1 ] || exit 1
[ $rc -eq 0 ] || { cat $OUT; exit 0; }
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'])"; }
for rep in 1 2 3 4; do
  for v in default lzbc; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_lazy_bcast_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
cat $OUT
)
;;
gpu_r05_session30)
(
# Round 5, GPU session 30: the lazy step reading the next code word at even steps only
# (MH_SMALL_LAZY_HALF=1, ab/lib_lzhalf.so: half the stage reads; wa changes only at a refill and
# no refill follows a refill). Decode tests through it, then the driver's frame command, default
# vs lzhalf, interleaved x 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_lazy_half_ab.txt
: > $OUT
MH_LIB=$GRAFT_REPO_ROOT/ab/lib_lzhalf.so timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_stress.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_lzhalf.log 2>&1
rc=$?
tail -2 gpurun_out/r05_pytest_lzhalf.log >> $OUT
[ $rc -le 1 ] || exit 1
[ $rc -eq 0 ] || { cat $OUT; exit 0; }
line() { python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_us', d['roofline']['kernel_us_avg'])"; }
for rep in 1 2 3 4; do
  for v in default lzhalf; do
    if [ "$v" = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
    r=$(timeout -k 10 150 python bench.py --workload frame --steps 20 --warmup 5 --no-extras --no-cpu-baseline 2>>gpurun_out/r05_lazy_half_ab.err) || { echo "$v FAILED" >> $OUT; exit 1; }
    echo "$v frame $(echo "$r" | line)" >> $OUT
  done
  echo "rep $rep done"
done
cat $OUT
)
;;
gpu_r05_session31)
(
# Round 5, GPU session 31: per-wave stamps with core-clock cycles of the final single-frame
# kernel (lazy refill, even-step next-word reads): bench-style cold shuffled frames and the warm
# natural frame.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/r05_final_stamps.txt
: > $OUT
export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_stampclk.so
{ echo "== final --cold"; timeout -k 10 180 python3 scripts/diag_stamps.py --cold --clock --tag _final 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
{ echo "== final warm (natural frame)"; timeout -k 10 180 python3 scripts/diag_stamps.py --clock --tag _final 2>&1 | grep -v amdgpu.ids; } >> $OUT || exit 1
cat $OUT
)
;;
*) echo "unknown session $1"; exit 2 ;;
esac

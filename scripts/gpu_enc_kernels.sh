# Batched GPU encoder, per-kernel device time under rocprofv3 --kernel-trace --stats, for the
# default library and ab/lib_<x>.so variants (diagnostic variants: MH_PROFILE_NO_CHECK=1).
#   bash scripts/gpu_enc_kernels.sh "default splitnohist" -> gpurun_out/enc_kernels.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/enc_kernels.txt
for rep in 1 2; do
  for l in ${1:-default}; do
    if [ $l = default ]; then env=""; elif [[ $l == *no* ]]; then env="MH_LIB=$PWD/ab/lib_$l.so MH_PROFILE_NO_CHECK=1"; else env="MH_LIB=$PWD/ab/lib_$l.so"; fi
    rm -rf gpurun_out/encprof_$l
    env $env timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/encprof_$l -o run -- python3 scripts/enc_batch_profile.py 64 8 > gpurun_out/encprof_$l.log 2>&1 || { tail -20 gpurun_out/encprof_$l.log; exit 1; }
    python3 - "$l" gpurun_out/encprof_$l >> gpurun_out/enc_kernels.txt <<'PY'
import csv, glob, re, sys
lib, d = sys.argv[1], sys.argv[2]
f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    m = re.search(r"(enc_\w+)", r["Name"])
    if m:
        print(f"{lib:12s} {m.group(1):24s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.2f} us")
PY
    grep "us/frame" gpurun_out/encprof_$l.log | head -1 | sed "s/^/$l  /" >> gpurun_out/enc_kernels.txt
  done
done
cat gpurun_out/enc_kernels.txt

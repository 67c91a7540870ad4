# Timing of encoder variant libraries (gated async encode, BigBridge): default, then
# each ab/lib_<name>.so named in ENC_VARIANTS.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
for v in default ${ENC_VARIANTS}; do
  if [ $v = default ]; then unset MH_LIB; else export MH_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so; fi
  echo "== $v $(timeout -k 10 120 python3 scripts/enc_profile.py 256 2>&1 | grep 'gated' | tail -1)"
done
done

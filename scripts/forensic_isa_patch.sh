# Round-6 forensics (container side): code objects of round 5's spilled batch-kernel build,
# assembled from its device assembly unchanged and with one-instruction patches at the
# failing step, for scripts/forensic_isa_patch.py on the GPU box.
#   ab/isa_orig.hsaco  the build as compiled (commit 6793108's mh_decode.hip, no kernarg preload)
#   ab/isa_mov.hsaco   step 5's shift amount copied out of v79 first:
#                        v_mov_b32 v68, v79 ; v_lshrrev_b64 v[68:69], v68, v[50:51]
#   ab/isa_nop.hsaco   an s_nop 0 in front of the same shift (amount still in v79)
# Usage: bash scripts/forensic_isa_patch.sh <path of 6793108's mh_decode.hip>
set -euo pipefail
SRC=${1:?mh_decode.hip of commit 6793108}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/ab
TMP=$(mktemp -d)
LLVM=/opt/rocm/llvm/bin
mkdir -p "$OUT"
(cd "$(dirname "$SRC")" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC --cuda-device-only -S \
   -o "$TMP/orig.s" "$(basename "$SRC")" 2>/dev/null)
PAT='v_lshrrev_b64 v\[68:69\], v79, v\[50:51\]'
n=$(grep -c "$PAT" "$TMP/orig.s" || true)
[ "$n" = 1 ] || { echo "expected one shift with its amount in v79, found $n"; exit 1; }
sed "s/\t$PAT/\tv_mov_b32 v68, v79\n\tv_lshrrev_b64 v[68:69], v68, v[50:51]/" "$TMP/orig.s" > "$TMP/mov.s"
sed "s/\t$PAT/\ts_nop 0\n\tv_lshrrev_b64 v[68:69], v79, v[50:51]/" "$TMP/orig.s" > "$TMP/nop.s"
for v in orig mov nop; do
  $LLVM/clang --target=amdgcn-amd-amdhsa -mcpu=gfx950 -c "$TMP/$v.s" -o "$TMP/$v.o"
  $LLVM/ld.lld -shared "$TMP/$v.o" -o "$OUT/isa_$v.hsaco"
  echo "$OUT/isa_$v.hsaco"
done
diff "$TMP/orig.s" "$TMP/mov.s" || true
rm -rf "$TMP"

#!/bin/bash
# Build libsdmoe_hip_prev.so (the A/B baseline of tools/gpu_ab_lib.sh) from a git revision's csrc/ + include/,
# reusing this tree's object files for the sources that revision did not change. usage: bash tools/build_prev.sh [REV]
set -eu
REV=${1:-HEAD}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/sdmoe_prev.XXXXXX)
git -C "$R" archive "$REV" diffusion-models-moe_amd/csrc include | tar -x -C "$T"
mkdir -p "$T/diffusion-models-moe_amd/csrc/build"
for f in "$R"/diffusion-models-moe_amd/csrc/*.hip; do
  b=$(basename "$f" .hip)
  if cmp -s "$f" "$T/diffusion-models-moe_amd/csrc/$b.hip" && cmp -s "$R/include/sdmoe.h" "$T/include/sdmoe.h" \
     && cmp -s "$R/diffusion-models-moe_amd/csrc/common.h" "$T/diffusion-models-moe_amd/csrc/common.h" \
     && [ -f "$R/diffusion-models-moe_amd/csrc/build/$b.o" ]; then
    cp "$R/diffusion-models-moe_amd/csrc/build/$b.o" "$T/diffusion-models-moe_amd/csrc/build/"
  fi
done
touch "$T"/diffusion-models-moe_amd/csrc/build/*.o 2>/dev/null || true
make -C "$T/diffusion-models-moe_amd/csrc" -j8 LIB="$R/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_prev.so" > "$T/make.log" 2>&1 \
  || { tail -20 "$T/make.log"; exit 1; }
echo "built libsdmoe_hip_prev.so from $(git -C "$R" rev-parse --short "$REV")"
rm -rf "$T"

#!/bin/bash
# Build libsgm_hip.so from the sources of a git revision, for paired A/B
# timing against the working tree (tools/ab.sh).
# Usage: bash tools/variant_rev.sh REV NAME   -> build/NAME/libsgm_hip.so
set -e
REV=$1
NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/build/${NAME}_src
rm -rf "$SRC"
mkdir -p "$SRC" "$ROOT/build/$NAME"
git -C "$ROOT" archive "$REV" stereo_matching_amd/csrc include | tar -x -C "$SRC"
make -s -C "$SRC/stereo_matching_amd/csrc" -j8 OUT="$ROOT/build/$NAME/libsgm_hip.so" "$ROOT/build/$NAME/libsgm_hip.so" \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fno-honor-nans -mno-amdgpu-ieee -Wall -Wno-unused-result -I$SRC/include"
rm -rf "$SRC"
echo "built build/$NAME/libsgm_hip.so from $REV"

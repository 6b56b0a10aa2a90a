#!/bin/bash
# Build a variant of libsgm_hip.so from the current sources with extra
# compile flags, for paired A/B timing (tools/ab.sh).
# Usage: bash tools/variant.sh NAME "-DFLAG=1 ..."   -> build/NAME/libsgm_hip.so
set -e
NAME=$1
FLAGS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/build/${NAME}_src
rm -rf "$SRC"
mkdir -p "$SRC" "$ROOT/build/$NAME"
cp "$ROOT"/stereo_matching_amd/csrc/*.hip "$ROOT"/stereo_matching_amd/csrc/*.h "$ROOT"/stereo_matching_amd/csrc/Makefile "$SRC"/
make -s -C "$SRC" -j8 OUT="$ROOT/build/$NAME/libsgm_hip.so" "$ROOT/build/$NAME/libsgm_hip.so" \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fno-honor-nans -mno-amdgpu-ieee -Wall -Wno-unused-result -I$ROOT/include $FLAGS"
rm -f "$SRC"/*.o
echo "built build/$NAME/libsgm_hip.so ($FLAGS)"

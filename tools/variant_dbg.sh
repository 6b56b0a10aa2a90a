#!/bin/bash
# build a debug-library variant: vdbg.sh NAME "FLAGS"
set -e
NAME=$1; FLAGS=$2; ROOT=$(cd "$(dirname "$0")/.." && pwd); SRC=$ROOT/build/${NAME}_src
rm -rf $SRC; mkdir -p $SRC $ROOT/build/$NAME
cp $ROOT/stereo_matching_amd/csrc/*.hip $ROOT/stereo_matching_amd/csrc/*.h $ROOT/stereo_matching_amd/csrc/Makefile $SRC/
make -s -C $SRC -j8 DBG_OUT=$ROOT/build/$NAME/libsgm_hip_slantdbg.so $ROOT/build/$NAME/libsgm_hip_slantdbg.so \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fno-honor-nans -mno-amdgpu-ieee -Wall -Wno-unused-result -I$ROOT/include $FLAGS"
rm -rf $SRC
echo built $NAME

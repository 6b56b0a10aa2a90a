#!/bin/bash
# Instrumented build of libsgm_hip.so (-DSGM_STAMPS) into build/stamps/, for
# tools/stamps.py and tools/sky_stamps.py (load it with SGM_HIP_LIB).
set -e
cd "$(dirname "$0")/../stereo_matching_amd/csrc"
OUT=../../build/stamps
mkdir -p $OUT
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fno-honor-nans -mno-amdgpu-ieee -I../../include -DSGM_STAMPS"
for f in sgm_cost sgm_sweep sgm_pair sgm_post sgm_lk sgm_sky sgm_bm sgm_consumers sgm_capi; do
  /opt/rocm/bin/hipcc $FLAGS -c $f.hip -o $OUT/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libsgm_hip.so $OUT/*.o

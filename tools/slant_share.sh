#!/bin/bash
# The top-down slanted pass's share of the CUs beside the H pair (sgm_capi.hip
# slant_down_grid_eighths), swept on the debug build (SGM_SLANT_DOWN_EIGHTHS).
# Usage (GPU box): bash tools/slant_share.sh CONFIG REPS "EIGHTHS..."
set -o pipefail
CFG=$1; REPS=$2; SHARES=$3
mkdir -p gpurun_out
for r in $(seq 1 $REPS); do
  for e in $SHARES; do
    SGM_HIP_LIB=stereo_matching_amd/libsgm_hip_slantdbg.so SGM_SLANT_DOWN_EIGHTHS=$e \
      timeout -k 10 120 python bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline \
      > gpurun_out/share_last.json 2>> gpurun_out/share.err || { echo "bench failed ($e)"; tail -20 gpurun_out/share.err; exit 1; }
    python -c "
import json; r=json.loads(open('gpurun_out/share_last.json').read().strip().splitlines()[-1]); k=r['kernels']
print('$CFG eighths=$e %7.3f ms  down||h %.0f  down %.0f  hpair %.0f  up %.0f us' % (r['ms_per_step'], k['slant_down_hpair']['avg_us'], k['slant_down']['avg_us'], k['stage_a_h']['avg_us'], k['slant_up']['avg_us']))"
  done
done

#!/bin/bash
# round 6: the concurrent region with the dataflow top-down pass -- H pair
# issue priority x top-down share, paired against round 5's library
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
CFG=${1:-hd256}
run() {  # LIB EIGHTHS
  SGM_SLANT_DOWN_EIGHTHS=$2 SGM_HIP_LIB=$1 timeout -k 10 180 python bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/ab_last.json 2>> gpurun_out/ab.err || { echo "bench failed"; tail -5 gpurun_out/ab.err; exit 1; }
  python -c "
import json; r=json.loads(open('gpurun_out/ab_last.json').read().strip().splitlines()[-1]); k=r['kernels']
print('%-6s %-44s e=%s %8.3f ms  region %5.0f down %5.0f hpair %5.0f up %5.0f' % ('$CFG', '$1'[-44:], '$2', r['ms_per_step'], k['slant_down_hpair']['avg_us'], k['slant_down']['avg_us'], k['stage_a_h']['avg_us'], k['slant_up']['avg_us']))"
}
for rep in 1 2; do
  run build/base/libsgm_hip.so 7 || exit 1
  for L in stereo_matching_amd/libsgm_hip_slantdbg.so build/hp2/libsgm_hip_slantdbg.so build/hp3/libsgm_hip_slantdbg.so; do
    for e in 4 6 8; do run $L $e || exit 1; done
  done
done

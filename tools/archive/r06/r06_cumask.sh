#!/bin/bash
# round 6: the concurrent region on disjoint CU halves (hipExtStreamCreateWithCUMask), paired
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
DBG=stereo_matching_amd/libsgm_hip_slantdbg.so
run() {  # CFG MASK
  if [ "$2" == "none" ]; then unset SGM_SLANT_CUMASK; else export SGM_SLANT_CUMASK=$2; fi
  SGM_HIP_LIB=$DBG timeout -k 10 180 python bench.py --config $1 --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/ab_last.json 2>> gpurun_out/ab.err || { echo "bench failed"; tail -5 gpurun_out/ab.err; exit 1; }
  python -c "
import json; r=json.loads(open('gpurun_out/ab_last.json').read().strip().splitlines()[-1]); k=r['kernels']
print('%-6s mask=%-5s %8.3f ms  region %5.0f down %5.0f hpair %5.0f up %5.0f' % ('$1', '$2', r['ms_per_step'], k['slant_down_hpair']['avg_us'], k['slant_down']['avg_us'], k['stage_a_h']['avg_us'], k['slant_up']['avg_us']))"
}
run hd256 none > /dev/null || exit 1
for rep in 1 2 3; do for m in none even half; do run hd256 $m || exit 1; done; done
for rep in 1; do for m in none even half; do run 4k256 $m || exit 1; done; done

#!/bin/bash
# slant_up time per library variant (timing probes; results of probes are wrong)
set -o pipefail
CFG=${1:-hd256}; shift
for v in "$@"; do
  lib=stereo_matching_amd/libsgm_hip.so; [ "$v" != base ] && lib=build/$v/libsgm_hip.so
  SGM_SLANT=1 SGM_HIP_LIB=$lib timeout -k 10 300 python bench.py --config $CFG --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/probe_${CFG}_$v.json 2>/dev/null || exit 1
  python3 -c "
import json; r=json.load(open('gpurun_out/probe_${CFG}_$v.json')); k=r['kernels']
print('%-10s %-8s step %8.3f ms  slant_up %8.1f us' % ('$CFG', '$v', r['ms_per_step'], k['slant_up']['avg_us']), 'down %8.1f' % k.get('slant_down',{}).get('avg_us',0))"
done

#!/bin/bash
# round 6: row chains in the slanted passes -- hop-latency variants, paired
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # CFG LIB H
  SGM_SLANT_H=$3 SGM_HIP_LIB=$2 timeout -k 10 180 python bench.py --config $1 --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/ab_last.json 2>> gpurun_out/ab.err || { echo "bench failed"; tail -5 gpurun_out/ab.err; exit 1; }
  python -c "
import json; r=json.loads(open('gpurun_out/ab_last.json').read().strip().splitlines()[-1])
print('%-6s %-34s H=%s %8.3f ms  ' % ('$1', '$2'[-34:], '$3', r['ms_per_step']) + ' '.join('%s=%.0f' % (k[:10], v['share_per_step_ms'] * 1e3) for k, v in r['kernels'].items()))"
}
for cfg in hd256 4k256; do
  for rep in 1 2; do
    run $cfg stereo_matching_amd/libsgm_hip.so 0 || exit 1
    run $cfg stereo_matching_amd/libsgm_hip.so 1 || exit 1
    run $cfg build/hprio/libsgm_hip.so 1 || exit 1
    run $cfg build/hbusy/libsgm_hip.so 1 || exit 1
    run $cfg build/hnowait/libsgm_hip.so 1 || exit 1
  done
done

#!/bin/bash
# A/B of the slanted schedule (SGM_SLANT=0/1) on the big configs; per-kernel times
set -o pipefail
TAG=${1:-ab}
shift
for c in ${@:-hd256 4k256}; do
  for m in 0 1; do
    SGM_SLANT=$m timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline \
      > gpurun_out/${TAG}_${c}_slant$m.json 2> gpurun_out/${TAG}_${c}_slant$m.err || exit 1
    python3 -c "
import json; r=json.load(open('gpurun_out/${TAG}_${c}_slant$m.json'))
print('$c', 'slant=$m', r['value'], 'MPD/s', r['ms_per_step'], 'ms')
for k,v in sorted(r['kernels'].items(), key=lambda x:-x[1]['share_per_step_ms']): print('   %-22s %4d %10.1f us  %8.3f ms/step' % (k, v['launches'], v['avg_us'], v['share_per_step_ms']))"
  done
done

#!/bin/bash
# Paired A/B timing of one environment switch on one box: bench.py alternates
# between the values REPS times.  Usage (GPU box):
#   bash tools/ab_env.sh CONFIG REPS VAR VALUE_A VALUE_B [VALUE_C ...]
set -o pipefail
CFG=$1; REPS=$2; VAR=$3; shift 3
mkdir -p gpurun_out
for r in $(seq 1 $REPS); do
  for X in "$@"; do
    env $VAR=$X timeout -k 10 180 python bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline \
      > gpurun_out/ab_last.json 2>> gpurun_out/ab.err || { echo "bench failed for $VAR=$X"; tail -20 gpurun_out/ab.err; exit 1; }
    python -c "
import json; r=json.loads(open('gpurun_out/ab_last.json').read().strip().splitlines()[-1])
print('%-6s %s=%-4s %9.1f MPD/s %8.4f ms  ' % ('$CFG', '$VAR', '$X', r['value'], r['ms_per_step']) + ' '.join('%s=%.0f' % (k[:10], v['share_per_step_ms'] * 1e3) for k, v in r['kernels'].items()))"
  done
done

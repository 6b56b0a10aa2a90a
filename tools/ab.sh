#!/bin/bash
# Paired A/B timing of library builds on one box: bench.py alternates
# between the libraries REPS times (SGM_HIP_LIB), printing MPD/s and the
# per-kernel event time per step (us) of every run.  Usage (GPU box):
#   bash tools/ab.sh CONFIG REPS LIB_A LIB_B [LIB_C ...]
set -o pipefail
CFG=$1; REPS=$2; shift 2
mkdir -p gpurun_out
# one discarded run first: a fresh box runs its first seconds measurably
# faster than later ones (profiles/r06_experiments/r06l_tile_width.txt), which
# would favour whichever library ran first
SGM_HIP_LIB=$1 timeout -k 10 120 python bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline \
  > /dev/null 2>> gpurun_out/ab.err || { echo "warm-up bench failed"; tail -20 gpurun_out/ab.err; exit 1; }
for r in $(seq 1 $REPS); do
  for L in "$@"; do
    SGM_HIP_LIB=$L timeout -k 10 120 python bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline \
      > gpurun_out/ab_last.json 2>> gpurun_out/ab.err || { echo "bench failed for $L"; tail -20 gpurun_out/ab.err; exit 1; }
    python -c "
import json; r=json.loads(open('gpurun_out/ab_last.json').read().strip().splitlines()[-1])
print('%-28s %9.1f MPD/s %7.4f ms  ' % ('$L'[-28:], r['value'], r['ms_per_step']) + ' '.join('%s=%.1f' % (k[:10], v['share_per_step_ms'] * 1e3) for k, v in r['kernels'].items()))"
  done
done

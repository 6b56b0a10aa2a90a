#!/bin/bash
# Paired: frames on the handle's own stream (default) vs a caller's stream (--caller-stream).
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for a in "" "--caller-stream"; do
    timeout -k 10 120 python bench.py --steps 40 --warmup 4 --no-cpu-baseline --no-profile-pass $a > gpurun_out/r03_hsab.json 2>>gpurun_out/r03_hsab.err || exit 1
    python -c "
import json; r=json.loads(open('gpurun_out/r03_hsab.json').read().strip().splitlines()[-1]); print('k128 ${a:-handle-stream}', r['value'], r['ms_per_step'])"
  done
done
for a in "" "--caller-stream"; do
  timeout -k 10 120 python bench.py --config k128lr --steps 20 --warmup 3 --no-cpu-baseline --no-profile-pass $a > gpurun_out/r03_hsab.json 2>>gpurun_out/r03_hsab.err || exit 1
  python -c "
import json; r=json.loads(open('gpurun_out/r03_hsab.json').read().strip().splitlines()[-1]); print('k128lr ${a:-handle-stream}', r['value'], r['ms_per_step'])"
done

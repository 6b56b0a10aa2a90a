#!/bin/bash
# Run-to-run spread of the headline line on one box: 6 default runs (k128), 2 hd256.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3 4 5 6; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-profile-pass > gpurun_out/r03_spread.json 2>>gpurun_out/r03_spread.err || exit 1
  python -c "
import json; r=json.loads(open('gpurun_out/r03_spread.json').read().strip().splitlines()[-1]); print('k128', r['value'], r['ms_per_step'])"
done
for r in 1 2; do
  timeout -k 10 200 python bench.py --config hd256 --no-cpu-baseline --no-profile-pass > gpurun_out/r03_spread.json 2>>gpurun_out/r03_spread.err || exit 1
  python -c "
import json; r=json.loads(open('gpurun_out/r03_spread.json').read().strip().splitlines()[-1]); print('hd256', r['value'], r['ms_per_step'])"
done

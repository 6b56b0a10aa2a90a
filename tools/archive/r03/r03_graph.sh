#!/bin/bash
# Eager frames vs one captured HIP graph replayed per frame (bench.py --graph), paired runs.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
  for c in k128 k128lr; do
    for m in "" "--graph"; do
      timeout -k 10 300 python bench.py --config $c --no-cpu-baseline $m > gpurun_out/r03_graph.json 2>> gpurun_out/r03_graph.err || { tail -30 gpurun_out/r03_graph.err; exit 1; }
      python -c "
import json; r=json.loads(open('gpurun_out/r03_graph.json').read().strip().splitlines()[-1])
print('$c', '${m:-eager}', r['value'], r['ms_per_step'], r['roofline']['kernel_sum_ms_per_step'])"
    done
  done
done

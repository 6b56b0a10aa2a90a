#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for cfg in k128 k64; do
for r in 1 2; do
  for v in "cur 0" "cur 1" "nofix 1"; do
    set -- $v
    SGM_HIP_LIB=build/$1/libsgm_hip.so SGM_COSTH_SPLIT=$2 timeout -k 10 120 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_last.json 2>>gpurun_out/ab.err || exit 1
    python -c "
import json; r=json.loads(open('gpurun_out/ab_last.json').read().strip().splitlines()[-1])
print('$cfg $1 split=$2', r['ms_per_step'], 'cost_h', round(r['kernels']['cost_h']['share_per_step_ms']*1e3,1))"
  done
done
done
for w in 128 384 512; do
  SGM_HIP_LIB=build/cur/libsgm_hip.so SGM_COSTH_SPLIT=1 SGM_COSTH_WARM=$w timeout -k 10 120 python bench.py --config k128 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_last.json 2>>gpurun_out/ab.err || exit 1
  python -c "
import json; r=json.loads(open('gpurun_out/ab_last.json').read().strip().splitlines()[-1])
print('k128 warm=$w', r['ms_per_step'], 'cost_h', round(r['kernels']['cost_h']['share_per_step_ms']*1e3,1))"
done

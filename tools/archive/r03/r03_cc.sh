#!/bin/bash
# cc_count with saturating area adds: post filter parity, then the full-pipeline timings.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_post_filter.py tests/test_gpu_bm.py tests/test_example_node.py tests/test_gpu_real_texture.py \
  > gpurun_out/r03_cc_tests.log 2>&1 || { tail -40 gpurun_out/r03_cc_tests.log; exit 1; }
tail -1 gpurun_out/r03_cc_tests.log
for c in k128full 4k256full; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03_cc_$c.json || exit 1
  python -c "
import json; r=json.loads(open('gpurun_out/r03_cc_$c.json').read().strip().splitlines()[-1])
print('$c', r['value'], r['ms_per_step'], {k: round(v['share_per_step_ms']*1e3,1) for k, v in r['kernels'].items() if k.startswith('post') or k.startswith('lk') or k.startswith('sky')})"
done

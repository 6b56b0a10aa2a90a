#!/bin/bash
# Map-gather batching under torchrun (world 1 on one GPU), bench.py's default 20 steps: one
# collective per step vs one per G steps, with the single-process line for reference.
set -o pipefail
mkdir -p gpurun_out
run() {
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $1 bench.py --gpus 1 --no-cpu-baseline --no-profile-pass ${@:2} \
    > gpurun_out/r03_gather2.json 2>> gpurun_out/r03_gather2.err || exit 1
  python -c "
import json; r=json.loads(open('gpurun_out/r03_gather2.json').read().strip().splitlines()[-1])
print('${*:2}', r['value'], r['ms_per_step'])"
}
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile-pass > gpurun_out/r03_gather2.json || exit 1
  python -c "
import json; r=json.loads(open('gpurun_out/r03_gather2.json').read().strip().splitlines()[-1])
print('single-process', r['value'], r['ms_per_step'])"
  run 29611 --gather-every 1
  run 29612 --gather-every 2
  run 29613 --gather-every 4
  run 29614 --gather-every 5
  run 29615 --gather-every 10
done

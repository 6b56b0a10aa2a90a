#!/bin/bash
# Per-step cost of the map gather under torchrun (world 1 on one GPU): every step, every 4 steps,
# none (diagnostic), and the single-process line for reference.
set -o pipefail
mkdir -p gpurun_out
run() {
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $1 bench.py --gpus 1 --steps 40 --warmup 4 --no-cpu-baseline --no-profile-pass ${@:2} \
    > gpurun_out/r03_gather.json 2>> gpurun_out/r03_gather.err || exit 1
  python -c "
import json; r=json.loads(open('gpurun_out/r03_gather.json').read().strip().splitlines()[-1])
print('${*:2}', r['value'], r['ms_per_step'])"
}
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 4 --no-cpu-baseline --no-profile-pass > gpurun_out/r03_gather.json || exit 1
  python -c "
import json; r=json.loads(open('gpurun_out/r03_gather.json').read().strip().splitlines()[-1])
print('single-process', r['value'], r['ms_per_step'])"
  run 29601 --gather-every 1
  run 29602 --gather-every 4
  run 29603 --no-gather
done

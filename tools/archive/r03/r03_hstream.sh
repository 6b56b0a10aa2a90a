#!/bin/bash
# Bench on the handle's own stream: stream tests, bench lines, frame-boundary gap in the trace.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_schedules.py tests/test_gpu_distributed.py tests/test_capi.py > gpurun_out/r03_hs_tests.log 2>&1 \
  || { tail -40 gpurun_out/r03_hs_tests.log; exit 1; }
tail -1 gpurun_out/r03_hs_tests.log
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 40 --warmup 4 --no-cpu-baseline --no-profile-pass > gpurun_out/r03_hs.json || exit 1
  python -c "
import json; r=json.loads(open('gpurun_out/r03_hs.json').read().strip().splitlines()[-1]); print('k128', r['value'], r['ms_per_step'])"
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 1 --steps 40 --warmup 4 --no-cpu-baseline --no-profile-pass > gpurun_out/r03_hs.json 2>>gpurun_out/r03_hs.err || exit 1
python -c "
import json; r=json.loads(open('gpurun_out/r03_hs.json').read().strip().splitlines()[-1]); print('torchrun world1', r['value'], r['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_hs_prof -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-profile-pass > gpurun_out/r03_hs_prof.log 2>&1 || exit 1
python - <<'P'
import csv, glob
f = glob.glob('gpurun_out/r03_hs_prof/**/*kernel_trace.csv', recursive=True)[0]
seq = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:28]) for r in csv.DictReader(open(f)))
gaps = [((b[0] - a[1]) / 1000, a[2], b[2]) for a, b in zip(seq[-15:-1], seq[-14:])]
for g in gaps: print(f"{g[0]:6.2f} us {g[1]} -> {g[2]}")
P

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_schedules.py \
  tests/test_gpu_fullsize.py tests/test_gpu_fuzz.py > gpurun_out/r03_subcm2_tests.log 2>&1 || { tail -40 gpurun_out/r03_subcm2_tests.log; exit 1; }
tail -1 gpurun_out/r03_subcm2_tests.log
bash tools/ab_env.sh k128lr 3 SGM_SUB_CM 1 0 || exit 1
bash tools/ab_env.sh 4k256 2 SGM_SUB_CM 1 0 || exit 1

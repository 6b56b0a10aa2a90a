#!/bin/bash
# round 6: the H-wave slanted passes (SGM_SLANT_H=1): parity, then paired timing
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10"
SGM_SLANT_H=1 $T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py -k slant -m gpu > gpurun_out/r06_h1_fuzz.log 2>&1 || { tail -40 gpurun_out/r06_h1_fuzz.log; exit 1; }
tail -2 gpurun_out/r06_h1_fuzz.log
SGM_SLANT_H=1 $T 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_schedules.py tests/test_gpu_fullsize.py -k "slant or 1080 or 4k256_lr or schedules_agree" -m gpu > gpurun_out/r06_h1_full.log 2>&1 || { tail -40 gpurun_out/r06_h1_full.log; exit 1; }
tail -2 gpurun_out/r06_h1_full.log
bash tools/ab_env.sh hd256 2 SGM_SLANT_H 0 1 || exit 1
bash tools/ab_env.sh 4k256 1 SGM_SLANT_H 0 1 || exit 1

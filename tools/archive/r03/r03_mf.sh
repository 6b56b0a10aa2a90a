#!/bin/bash
# Median fill tile height (SGM_MF_ROWS 8 vs 16): parity under both, then paired timing.
set -o pipefail
mkdir -p gpurun_out
for R in 4 8; do
  SGM_MF_ROWS=$R timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_post_filter.py tests/test_gpu_real_texture.py tests/test_example_node.py \
    > gpurun_out/r03_mf_tests_$R.log 2>&1 || { tail -40 gpurun_out/r03_mf_tests_$R.log; exit 1; }
  echo "rows $R: $(tail -1 gpurun_out/r03_mf_tests_$R.log)"
done
bash tools/ab_env.sh k128full 3 SGM_MF_ROWS 4 8 16 || exit 1
bash tools/ab_env.sh 4k256full 1 SGM_MF_ROWS 4 8 16 || exit 1

#!/bin/bash
# round 6: hang-guard records at D = 64 and 256, and the default bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for D in 64 256; do
  timeout -k 10 170 python tools/slant_guard.py --D $D > gpurun_out/r06_guard_d$D.log 2>&1 || { tail -20 gpurun_out/r06_guard_d$D.log; exit 1; }
  grep "^{" gpurun_out/r06_guard_d$D.log | tail -1 > gpurun_out/r06_slant_guard_d$D.json
  cat gpurun_out/r06_slant_guard_d$D.json
done
timeout -k 10 300 python bench.py > gpurun_out/r06_bench_default.json 2> gpurun_out/r06_bench_default.err || { tail -20 gpurun_out/r06_bench_default.err; exit 1; }
cat gpurun_out/r06_bench_default.json

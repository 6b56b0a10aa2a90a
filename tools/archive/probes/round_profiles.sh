#!/bin/bash
# Round-end evidence: all bench configs, rocprof kernel stats of the default
# (k128) and full (k128full) benches.  Usage: bash tools/round_profiles.sh TAG
set -o pipefail
TAG=${1:-dev}
bash tools/bench_all.sh $TAG > gpurun_out/${TAG}_bench_all.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench_all.log; exit 1; }
head -6 gpurun_out/${TAG}_bench_all.log
bash tools/prof_full.sh $TAG k128 | tail -3 || exit 1
bash tools/prof_full.sh $TAG 4k256 | tail -3 || exit 1

#!/bin/bash
# Round-3 evidence on the shipped code: every bench config, rocprof kernel
# stats per config, PMC FETCH/WRITE passes per config tagged with the commit.
# Usage (GPU box): GIT_SHA=<commit> bash tools/r03_round.sh TAG [bench|prof|pmc]...
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
for part in "$@"; do
  case $part in
  bench)
    for c in k128 k64 k128lr k128full hd256 4k256 4k256full; do
      timeout -k 10 300 python bench.py --config $c > gpurun_out/${TAG}_bench_$c.json 2>> gpurun_out/${TAG}_bench.err || { echo "bench $c failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
      python -c "
import json; r=json.loads(open('gpurun_out/${TAG}_bench_$c.json').read().strip().splitlines()[-1])
print('$c', r['value'], 'MPD/s', r['ms_per_step'], 'ms', 'roof', r['roofline']['kernel'], r['roofline']['frac'], 'cpu', (r['cpu_baseline'] or {}).get('value'))"
    done ;;
  prof)
    for c in k128 k128lr hd256 4k256 k128full; do
      bash tools/prof_full.sh $TAG $c | tail -2 || exit 1
    done ;;
  pmc)
    for c in k128 k64 k128lr hd256 4k256 k128full 4k256full; do
      bash tools/pmc.sh $TAG $c > gpurun_out/${TAG}_pmc_$c.txt 2>&1 || { tail -20 gpurun_out/${TAG}_pmc_$c.txt; exit 1; }
      echo "pmc $c done"
    done ;;
  esac
done

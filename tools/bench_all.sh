#!/bin/bash
# All bench configs + rocprof kernel stats of the full K128 pipeline.
# Usage (on the GPU box, via gpurun): bash tools/bench_all.sh TAG
set -o pipefail
TAG=${1:-dev}
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in k128 k128lr k128full hd256 4k256 4k256full; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/${TAG}_bench_$c.json 2>> gpurun_out/${TAG}_bench.err || { echo "bench $c failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
  python -c "
import json,sys; r=json.loads(open('gpurun_out/${TAG}_bench_$c.json').read().strip().splitlines()[-1])
print('$c', r['value'], 'MPD/s', r['ms_per_step'], 'ms', 'roof', r['roofline']['kernel'], r['roofline']['frac'], 'cpu', (r['cpu_baseline'] or {}).get('value'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_proffull -o run --output-format csv -- python bench.py --config k128full --steps 10 --no-cpu-baseline --no-profile-pass > gpurun_out/${TAG}_proffull.log 2>&1 || { tail -20 gpurun_out/${TAG}_proffull.log; exit 1; }
python - "$TAG" <<'PY'
import csv, sys
tag = sys.argv[1]
for row in csv.DictReader(open(f"gpurun_out/{tag}_proffull/run_kernel_stats.csv")):
    print("  %-60s %4s %10.1f us" % (row["Name"][:60], row["Calls"], float(row["AverageNs"]) / 1e3))
PY

#!/bin/bash
# rocprofv3 kernel stats of one bench config (default: the full K128 pipeline).
# Usage (on the GPU box): bash tools/prof_full.sh TAG [config]
set -o pipefail
TAG=${1:-dev}; CFG=${2:-k128full}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_${CFG} -o run --output-format csv -- python bench.py --config $CFG --steps 10 --no-cpu-baseline --no-profile-pass > gpurun_out/${TAG}_prof_${CFG}.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof_${CFG}.log; exit 1; }
python - "$TAG" "$CFG" <<'PY'
import csv, sys
tag, cfg = sys.argv[1], sys.argv[2]
tot = 0.0
for row in csv.DictReader(open(f"gpurun_out/{tag}_prof_{cfg}/run_kernel_stats.csv")):
    tot += float(row["TotalDurationNs"])
    print("  %-60s %4s %10.1f us" % (row["Name"][:60], row["Calls"], float(row["AverageNs"]) / 1e3))
print("total kernel time per call of bench step: %.1f us" % (tot / 13 / 1e3))
PY

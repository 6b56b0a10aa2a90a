#!/bin/bash
# Do the TCC "DRAM" request counters tell Infinity Cache hits from HBM?  One pass with the
# read/write request totals and their DRAM-destined parts (4 TCC counters), kernel trace only.
# Usage (GPU box): bash tools/pmc_dram.sh TAG [config]
set -o pipefail
TAG=${1:-dev}; CFG=${2:-k128}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum \
  --kernel-trace -d gpurun_out/${TAG}_dram -o run --output-format csv \
  -- python bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass \
  > gpurun_out/${TAG}_dram.log 2>&1 || { tail -20 gpurun_out/${TAG}_dram.log; exit 1; }
python - "$TAG" <<'P'
import csv, glob, sys
from collections import defaultdict
sys.path.insert(0, "tools")
from pmc_reduce import short
tag = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"gpurun_out/{tag}_dram/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[short(r["Kernel_Name"]) or r["Kernel_Name"][:30]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(f"{k:22s} " + "  ".join(f"{c.replace('TCC_EA0_', '')}={sum(v)/len(v):.4g}" for c, v in sorted(cs.items())))
P

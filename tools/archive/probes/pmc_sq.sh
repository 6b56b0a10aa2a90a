#!/bin/bash
# Stall breakdown per kernel from SQ / TCC counters (one rocprofv3 pass per
# counter group, kernel trace only).  Usage (GPU box): bash tools/pmc_sq.sh TAG
set -o pipefail
TAG=${1:-dev}
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -f gpurun_out/counters_list.txt ] || timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES"
G2="TCC_HIT_sum TCC_MISS_sum SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES"
i=0
for G in "$G1" "$G2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $G --kernel-trace -d gpurun_out/${TAG}_sq$i -o run --output-format csv \
    -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile-pass \
    > gpurun_out/${TAG}_sq$i.log 2>&1 || { tail -20 gpurun_out/${TAG}_sq$i.log; exit 1; }
done
python - "$TAG" <<'PY'
import csv, glob, sys
from collections import defaultdict
tag = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"gpurun_out/{tag}_sq*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void sgm::", "")[:40]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print(k)
    print("   " + "  ".join(f"{c}={m[c]:.4g}" for c in sorted(m)))
PY

#!/bin/bash
# Per-kernel counter means for arbitrary counter groups, one rocprofv3 pass
# per group (kernel trace only).  Usage (GPU box):
#   bash tools/pmc_groups.sh TAG "CNT_A CNT_B ..." ["CNT_C ..."] ...
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for G in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $G --kernel-trace -d gpurun_out/${TAG}_g$i -o run --output-format csv \
    -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile-pass \
    > gpurun_out/${TAG}_g$i.log 2>&1 || { tail -20 gpurun_out/${TAG}_g$i.log; exit 1; }
done
python - "$TAG" <<'PY'
import csv, glob, sys
from collections import defaultdict
tag = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"gpurun_out/{tag}_g*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void sgm::", "")[:40]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print(k)
    print("   " + "  ".join(f"{c}={m[c]:.4g}" for c in sorted(m)))
PY

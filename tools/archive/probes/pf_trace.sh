#!/bin/bash
# Per-launch durations of the post-filter kernels (rocprofv3 kernel trace).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pftrace -o run -- python tools/pf_probe.py quick > gpurun_out/pftrace.log 2>&1 || { tail -20 gpurun_out/pftrace.log; exit 1; }
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/pftrace/**/run_kernel_trace.csv", recursive=True) + glob.glob("gpurun_out/pftrace/run_kernel_trace.csv")
rows = list(csv.DictReader(open(f[0])))
for r in rows:
    n = r["Kernel_Name"]
    if "median" in n or "cc_" in n:
        print("%-28s %8.1f us" % (n.split("(")[0].split("::")[-1][:28], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
PY

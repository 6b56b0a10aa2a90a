#!/bin/bash
# GPU round trip used during development: parity tests, bench, rocprof stats.
# Usage (on the GPU box, via gpurun): bash tools/gpu_check.sh TAG [full]
set -o pipefail
TAG=${1:-dev}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_cpp_surface.py -m gpu -x -q > gpurun_out/${TAG}_parity.log 2>&1 || { tail -30 gpurun_out/${TAG}_parity.log; exit 1; }
tail -2 gpurun_out/${TAG}_parity.log
if [ "$2" == "full" ]; then
  timeout -k 10 900 python -m pytest tests/test_gpu_fullsize.py -x -q > gpurun_out/${TAG}_full.log 2>&1 || { tail -30 gpurun_out/${TAG}_full.log; exit 1; }
  tail -2 gpurun_out/${TAG}_full.log
fi
timeout -k 10 300 python bench.py --host-io > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
timeout -k 10 300 python bench.py --config k128lr --no-cpu-baseline > gpurun_out/${TAG}_bench_lr.json 2>> gpurun_out/${TAG}_bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py --steps 10 --no-cpu-baseline --no-profile-pass > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python - "$TAG" <<'PY'
import csv, json, sys
tag = sys.argv[1]
for f in (f"gpurun_out/{tag}_bench.json", f"gpurun_out/{tag}_bench_lr.json"):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    print(r["config"]["views"], "views:", r["value"], "MPD/s", r["ms_per_step"], "ms/step", "roofline", r["roofline"]["kernel"], r["roofline"]["frac"])
    print("   ", {k: v["avg_us"] for k, v in r["kernels"].items()})
for row in csv.DictReader(open(f"gpurun_out/{tag}_prof/run_kernel_stats.csv")):
    print("  %-60s %4s %10.1f us" % (row["Name"][:60], row["Calls"], float(row["AverageNs"]) / 1e3))
PY

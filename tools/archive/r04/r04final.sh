# round-4 final evidence on the shipped sources: GPU suite, smoke, benches, rocprof, PMC
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04f_pytest_gpu.log 2>&1; tail -2 gpurun_out/r04f_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04f_smoke.log 2>&1; tail -1 gpurun_out/r04f_smoke.log
GIT_SHA=$1 bash tools/round.sh r04f bench prof pmc || exit 1
cp profiles/pmc_traffic.json gpurun_out/r04f_pmc_traffic_all.json
for c in hd256 4k256 4k256full; do echo "$c: $(python tools/trace_span.py gpurun_out/r04f_prof_$c/run_kernel_trace.csv | head -1)"; done

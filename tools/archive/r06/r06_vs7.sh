set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06c_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r06c_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06c_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r06c_smoke.log

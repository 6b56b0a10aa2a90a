timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04k_pytest_gpu.log 2>&1; tail -3 gpurun_out/r04k_pytest_gpu.log
GIT_SHA=$1 bash tools/round.sh r04k bench

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_vstrip.py tests/test_gpu_fuzz.py tests/test_gpu_schedules.py -k "vstrip or slant or right_view or strips" -x -q --timeout 200 --timeout-method thread > gpurun_out/vs10_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/vs10_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config 4k256full > gpurun_out/vs10_4k256full.json 2> gpurun_out/vs10_bench.err || exit $?
tail -1 gpurun_out/vs10_4k256full.json | cut -c1-300

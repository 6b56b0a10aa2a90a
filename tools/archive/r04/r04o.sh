timeout -k 10 120 python -u tools/dbg/slant_check.py > gpurun_out/slant7.log 2>&1; tail -1 gpurun_out/slant7.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_graph.py tests/test_gpu_schedules.py tests/test_gpu_fuzz.py tests/test_gpu_fullsize.py tests/test_gpu_threads.py > gpurun_out/r04o_tests.log 2>&1; tail -2 gpurun_out/r04o_tests.log
bash tools/slant_ab.sh r04o hd256 4k256

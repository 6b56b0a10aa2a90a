timeout -k 10 120 python -u tools/dbg/slant_check.py > gpurun_out/slant8.log 2>&1; tail -1 gpurun_out/slant8.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fuzz.py tests/test_gpu_schedules.py tests/test_gpu_graph.py -k "slant or default or replays" > gpurun_out/r04p_tests.log 2>&1; tail -1 gpurun_out/r04p_tests.log
bash tools/ab.sh hd256 2 build/prev/libsgm_hip.so stereo_matching_amd/libsgm_hip.so
bash tools/ab.sh 4k256 1 build/prev/libsgm_hip.so stereo_matching_amd/libsgm_hip.so

set -o pipefail
N=stereo_matching_amd/libsgm_hip.so
P=build/prev/libsgm_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_graph.py tests/test_gpu_threads.py tests/test_gpu_fuzz.py -x -q --timeout 200 --timeout-method thread > gpurun_out/calt_pytest.log 2>&1 || { tail -20 gpurun_out/calt_pytest.log; exit 1; }
bash tools/ab.sh k128 4 $P $N > gpurun_out/calt_k128.txt 2>&1 || exit 1
bash tools/ab.sh k128full 1 $P $N > gpurun_out/calt_k128full.txt 2>&1 || exit 1

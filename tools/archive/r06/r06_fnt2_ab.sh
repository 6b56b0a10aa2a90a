set -o pipefail
N=stereo_matching_amd/libsgm_hip.so
P=build/prev/libsgm_hip.so
bash tools/ab.sh k128lr 3 $P $N > gpurun_out/fnt2_k128lr.txt 2>&1 || exit 1
bash tools/ab.sh k128full 2 $P $N > gpurun_out/fnt2_k128full.txt 2>&1 || exit 1
bash tools/ab.sh k128 3 $P $N > gpurun_out/fnt2_k128.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -k "1242" > gpurun_out/fnt2_pytest.log 2>&1

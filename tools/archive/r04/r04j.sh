# exit states stored by the compute waves (no publisher wave): parity, stamps, A/B
timeout -k 10 120 python -u tools/dbg/slant_check.py > gpurun_out/slant5.log 2>&1; tail -1 gpurun_out/slant5.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fuzz.py -k slant > gpurun_out/slant_fuzz.log 2>&1; tail -1 gpurun_out/slant_fuzz.log
SGM_HIP_LIB=build/slantst/libsgm_hip.so timeout -k 10 100 python tools/slant_stamps.py 1080 1920 256 2 || exit 1
SGM_HIP_LIB=build/slantst/libsgm_hip.so timeout -k 10 100 python tools/slant_stamps.py 2160 3840 256 2 || exit 1
bash tools/slant_ab.sh r04j hd256 4k256 || exit 1

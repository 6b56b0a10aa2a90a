bash tools/dbg/slant_grid.sh
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fuzz.py -k slant > gpurun_out/slant_fuzz.log 2>&1; tail -2 gpurun_out/slant_fuzz.log
SGM_HIP_LIB=build/slantst/libsgm_hip.so timeout -k 10 100 python tools/slant_stamps.py 2160 3840 256 2
bash tools/slant_probe.sh hd256 base && bash tools/slant_probe.sh 4k256 base

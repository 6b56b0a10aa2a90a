# stamps (per-tile accumulation), slant vs banded A/B, full GPU suite
SGM_HIP_LIB=build/slantst/libsgm_hip.so timeout -k 10 100 python tools/slant_stamps.py 2160 3840 256 2 || exit 1
SGM_HIP_LIB=build/slantst/libsgm_hip.so timeout -k 10 100 python tools/slant_stamps.py 1080 1920 256 2 || exit 1
bash tools/slant_ab.sh r04i hd256 4k256 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04i_pytest_gpu.log 2>&1; tail -3 gpurun_out/r04i_pytest_gpu.log

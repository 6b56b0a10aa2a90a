# slant parity + timing (branch-free receiver, deferred WTA), final-pass XCD column map A/B + PMC
timeout -k 10 120 python -u tools/dbg/slant_check.py > gpurun_out/slant3.log 2>&1; tail -1 gpurun_out/slant3.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fuzz.py -k slant > gpurun_out/slant_fuzz.log 2>&1; tail -1 gpurun_out/slant_fuzz.log
SGM_HIP_LIB=build/slantst/libsgm_hip.so timeout -k 10 100 python tools/slant_stamps.py 2160 3840 256 2
bash tools/slant_probe.sh hd256 base wtainl pnocour && bash tools/slant_probe.sh 4k256 base wtainl pnocour
bash tools/ab.sh k128 3 build/noxcd/libsgm_hip.so stereo_matching_amd/libsgm_hip.so
GIT_SHA=wip bash tools/pmc.sh r04x k128

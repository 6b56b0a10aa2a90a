# granules in access order: parity, A/B, PMC at 4K
timeout -k 10 120 python -u tools/dbg/slant_check.py > gpurun_out/slant6.log 2>&1; tail -1 gpurun_out/slant6.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fuzz.py tests/test_gpu_schedules.py > gpurun_out/slant_fuzz.log 2>&1; tail -1 gpurun_out/slant_fuzz.log
bash tools/slant_ab.sh r04l hd256 4k256 || exit 1
bash tools/pmc.sh r04l 4k256 > gpurun_out/r04l_pmc_4k256.txt 2>&1; tail -8 gpurun_out/r04l_pmc_4k256.txt

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_vstrip.py tests/test_gpu_fuzz.py -k "vstrip or slant" -x -q --timeout 200 --timeout-method thread > gpurun_out/vs8_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/vs8_pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=3 timeout -k 10 400 python -u tools/vstrip_ab.py 1080x1920x256x2 1080x1920x128x2 2160x3840x256x2 > gpurun_out/vs8_ab.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/vs8_ab.txt

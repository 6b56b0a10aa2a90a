set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_vstrip.py -x -q --timeout 200 --timeout-method thread > gpurun_out/vs1_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/vs1_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/vstrip_ab.py 1080x1920x256x2 2160x3840x256x2 1080x1920x128x2 > gpurun_out/vs1_ab.txt 2>&1
rc=$?
cat gpurun_out/vs1_ab.txt | grep -v amdgpu.ids
exit $rc

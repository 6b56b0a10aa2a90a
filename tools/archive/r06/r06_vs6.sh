set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_vstrip.py -x -q --timeout 200 --timeout-method thread > gpurun_out/vs6_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/vs6_pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=2 timeout -k 10 300 python -u tools/vstrip_ab.py 1080x1920x256x2 1080x1920x128x2 2160x3840x256x2 > gpurun_out/vs6_ab.txt 2>&1 || exit $?
for v in pd4 ck0; do
echo "== $v" >> gpurun_out/vs6_ab.txt
SGM_HIP_LIB=$PWD/build/$v/libsgm_hip_slantdbg.so REPS=2 timeout -k 10 300 python -u tools/vstrip_ab.py 1080x1920x256x2 1080x1920x128x2 2160x3840x256x2 >> gpurun_out/vs6_ab.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/vs6_ab.txt

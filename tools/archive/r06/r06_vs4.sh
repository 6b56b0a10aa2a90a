set -o pipefail
mkdir -p gpurun_out
for v in nc16 nc16nost; do
  echo "== $v" >> gpurun_out/vs4_ab.txt
  SGM_HIP_LIB=$PWD/build/$v/libsgm_hip_slantdbg.so REPS=2 timeout -k 10 300 python -u tools/vstrip_ab.py 1080x1920x256x2 1080x1920x128x2 2160x3840x256x2 >> gpurun_out/vs4_ab.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/vs4_ab.txt

set -o pipefail
mkdir -p gpurun_out
for v in nost noh nov noraw; do
  echo "== $v" >> gpurun_out/vs3_ab.txt
  SGM_HIP_LIB=$PWD/build/$v/libsgm_hip_slantdbg.so REPS=1 timeout -k 10 300 python -u tools/vstrip_ab.py 1080x1920x256x2 1080x1920x128x2 >> gpurun_out/vs3_ab.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/vs3_ab.txt | grep -v twopass

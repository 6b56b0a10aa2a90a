set -o pipefail
B=stereo_matching_amd/libsgm_hip.so
bash tools/ab.sh hd256 3 $B build/hnt/libsgm_hip.so > gpurun_out/hnt_hd256.txt 2>&1 || exit 1
bash tools/ab.sh 4k256 2 $B build/hnt/libsgm_hip.so > gpurun_out/hnt_4k256.txt 2>&1 || exit 1
bash tools/ab.sh k128 2 $B build/hnt/libsgm_hip.so > gpurun_out/hnt_k128.txt 2>&1 || exit 1

set -o pipefail
B=stereo_matching_amd/libsgm_hip.so
bash tools/ab.sh k128 4 $B build/sb4/libsgm_hip.so build/vb4/libsgm_hip.so build/sb8vb8/libsgm_hip.so > gpurun_out/sb_k128.txt 2>&1 || exit 1
bash tools/ab.sh k64 2 $B build/sb4/libsgm_hip.so build/vb4/libsgm_hip.so build/sb8vb8/libsgm_hip.so > gpurun_out/sb_k64.txt 2>&1 || exit 1

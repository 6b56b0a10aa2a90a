set -o pipefail
B=stereo_matching_amd/libsgm_hip.so
bash tools/ab.sh k128 4 $B build/hb8/libsgm_hip.so build/hb16/libsgm_hip.so build/hb32/libsgm_hip.so build/hb8d4/libsgm_hip.so build/hb8d8/libsgm_hip.so > gpurun_out/hb_k128b.txt 2>&1 || exit 1

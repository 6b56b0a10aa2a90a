set -o pipefail
B=stereo_matching_amd/libsgm_hip.so
bash tools/ab.sh hd256 3 $B build/snt1/libsgm_hip.so build/snt2/libsgm_hip.so build/snt3/libsgm_hip.so > gpurun_out/snt_hd256.txt 2>&1 || exit 1
bash tools/ab.sh 4k256 2 $B build/snt1/libsgm_hip.so build/snt2/libsgm_hip.so build/snt3/libsgm_hip.so > gpurun_out/snt_4k256.txt 2>&1 || exit 1

set -o pipefail
B=stereo_matching_amd/libsgm_hip.so
bash tools/ab.sh k128 4 $B build/fnt/libsgm_hip.so build/l8nt/libsgm_hip.so build/both/libsgm_hip.so > gpurun_out/fnt_k128.txt 2>&1 || exit 1
bash tools/ab.sh k128lr 2 $B build/fnt/libsgm_hip.so build/l8nt/libsgm_hip.so build/both/libsgm_hip.so > gpurun_out/fnt_k128lr.txt 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")" > gpurun_out/r06z_smoke.log 2>&1

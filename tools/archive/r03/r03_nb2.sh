#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
bash tools/ab.sh hd256 2 build/nb3/libsgm_hip.so build/nb4/libsgm_hip.so || exit 1
bash tools/ab.sh 4k256 2 build/nb3/libsgm_hip.so build/nb4/libsgm_hip.so || exit 1

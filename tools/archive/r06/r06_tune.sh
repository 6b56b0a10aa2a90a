#!/bin/bash
# round 6: slanted-pass knobs re-tuned for the dataflow passes (paired)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L="stereo_matching_amd/libsgm_hip.so build/pw0/libsgm_hip.so build/rp2/libsgm_hip.so build/gap48/libsgm_hip.so build/r2/libsgm_hip.so build/dn12/libsgm_hip.so build/dn4/libsgm_hip.so"
bash tools/ab.sh hd256 3 $L || exit 1
bash tools/ab.sh 4k256 1 $L || exit 1

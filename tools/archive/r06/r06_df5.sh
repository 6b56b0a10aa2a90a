#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10 300"
PROF=1 REPS=1 $T python tools/slant_sweep.py "4" 1080x1920x256x2 || exit 1
SGM_HIP_LIB=stereo_matching_amd/libsgm_hip_slantdbg.so SGM_SLANT_DOWN_EIGHTHS=4 $T python bench.py --config hd256 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/b.json 2>gpurun_out/b.err || exit 1
python -c "
import json; r=json.loads(open('gpurun_out/b.json').read().strip().splitlines()[-1])
print('bench', r['ms_per_step'], {k: v['avg_us'] for k, v in r['kernels'].items()})"

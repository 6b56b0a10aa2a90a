bash tools/dbg/slant_grid.sh
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fuzz.py -k "test_random_frame and not banded and not slant" > gpurun_out/joint_fuzz.log 2>&1; tail -2 gpurun_out/joint_fuzz.log
for c in k64 k128lr; do timeout -k 10 200 python bench.py --config $c --steps 20 --no-cpu-baseline > gpurun_out/joint_$c.json 2>/dev/null && python3 -c "
import json; r=json.load(open('gpurun_out/joint_$c.json')); print('$c', r['value'], r['ms_per_step'], {k:v['avg_us'] for k,v in r['kernels'].items()})"; done

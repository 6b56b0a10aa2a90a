set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_post_filter.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pf_tests.log 2>&1 || { tail -40 gpurun_out/pf_tests.log; exit 1; }
tail -3 gpurun_out/pf_tests.log
timeout -k 10 300 python bench.py --config k128lr --post-filter --no-cpu-baseline > gpurun_out/pf_bench.json 2> gpurun_out/pf_bench.err || { tail -20 gpurun_out/pf_bench.err; exit 1; }
python -c "
import json; r=json.loads(open('gpurun_out/pf_bench.json').read().strip().splitlines()[-1])
print(r['value'], r['ms_per_step']); print({k:(v['launches'],v['avg_us']) for k,v in r['kernels'].items()}); print(r['roofline'].get('post_filter_ms_per_step'))"

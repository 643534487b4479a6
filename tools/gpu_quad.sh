set -e
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_w2.py > gpurun_out/quad_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "PASS|FAIL|Error|error" gpurun_out/quad_tests.log | tail -30; exit 1; }
tail -3 gpurun_out/quad_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/quad_bench.json 2> gpurun_out/quad_bench.err
python -c "
import json;d=json.loads(open('gpurun_out/quad_bench.json').read().strip().splitlines()[-1])
print({k:v for k,v in (d.get('extra') or {}).items() if 'plan' in k or 'c1' in k})"

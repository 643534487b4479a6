# GPU rehearsal of the round-end checks: the -m gpu suite, then a short bench with extras.
set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|error|assert" gpurun_out/gpu_tests.log | tail -30; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_short.json 2> gpurun_out/bench_short.err
python -c "
import json;d=json.loads(open('gpurun_out/bench_short.json').read().strip().splitlines()[-1])
print(d['value'], d['roofline']['frac'])
print({k:round(v,4) for k,v in (d.get('extra') or {}).items()})"

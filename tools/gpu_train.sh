# GPU check of the training step: its -m gpu tests, the GEMM probe, the bench's train extras.
set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_train.py > gpurun_out/train_tests.log 2>&1 || { tail -30 gpurun_out/train_tests.log; exit 1; }
tail -2 gpurun_out/train_tests.log
timeout -k 10 300 python -u tools/gemm_probe.py 20000 mfma > gpurun_out/gemm.json
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_short.json 2> gpurun_out/bench_short.err
python -c "
import json;d=json.loads(open('gpurun_out/bench_short.json').read().strip().splitlines()[-1])
print({k:round(v,3) for k,v in (d.get('extra') or {}).items() if 'train' in k})"

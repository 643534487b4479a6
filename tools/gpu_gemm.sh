# Training-GEMM check on one GPU: the GEMM / training parity tests, then the GEMM probe with
# the LDS panel kernel (default), the register-stream one (PNTF_GEMM_PANEL=1) and no panel
# path (=0), then the training-step timing with the first two.
set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_train.py > gpurun_out/gemm_tests.log 2>&1 || { tail -40 gpurun_out/gemm_tests.log; exit 1; }
tail -2 gpurun_out/gemm_tests.log
for m in 2 1 0; do
  PNTF_GEMM_PANEL=$m timeout -k 10 300 python -u tools/gemm_probe.py 20000 mfma > gpurun_out/gemm_probe_$m.json
  echo "panel mode $m"; python3 -c "
import json; d = json.load(open('gpurun_out/gemm_probe_$m.json'))
print({t: {k: v for k, v in r.items() if 'err' not in k} for t, r in d.items()})"
done
for m in 2 1; do
  PNTF_GEMM_PANEL=$m timeout -k 10 300 python -u tools/train_profile.py > gpurun_out/train_step_$m.log 2>&1 && tail -1 gpurun_out/train_step_$m.log
done

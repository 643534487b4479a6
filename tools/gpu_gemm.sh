# Training-GEMM check on one GPU: the GEMM / training parity tests, then the GEMM probe with
# the panel path on and off (PNTF_GEMM_PANEL=0), then the training-step timing.
set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_train.py > gpurun_out/gemm_tests.log 2>&1 || { tail -40 gpurun_out/gemm_tests.log; exit 1; }
tail -2 gpurun_out/gemm_tests.log
timeout -k 10 300 python -u tools/gemm_probe.py 20000 mfma > gpurun_out/gemm_probe_panel.json
PNTF_GEMM_PANEL=0 timeout -k 10 300 python -u tools/gemm_probe.py 20000 mfma > gpurun_out/gemm_probe_lds.json
cat gpurun_out/gemm_probe_panel.json gpurun_out/gemm_probe_lds.json
timeout -k 10 300 python -u tools/train_profile.py > gpurun_out/train_step.log 2>&1 && tail -5 gpurun_out/train_step.log
PNTF_GEMM_PANEL=0 timeout -k 10 300 python -u tools/train_profile.py > gpurun_out/train_step_lds.log 2>&1 && tail -2 gpurun_out/train_step_lds.log

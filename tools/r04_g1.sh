set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tests/diag/coexec32_probe > gpurun_out/r04_coexec32.txt 2>&1 || echo "probe rc=$?"
timeout -k 10 300 python -u -m pytest tests/test_out_grad.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04_outgrad.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/r04_outgrad.log; exit 1; }
timeout -k 10 800 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r04_bench0.log 2>&1

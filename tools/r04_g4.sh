set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_train.py -x -v --timeout 120 --timeout-method thread -k "ragged or k0 or fused_linear_act or loss_backward or adamw" > gpurun_out/r04_train_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/r04_train_tests.log; exit 1; }
timeout -k 10 300 python -u tools/train_sched_probe.py 10 > gpurun_out/r04_train_sched.txt 2>&1
timeout -k 10 200 python -u tests/diag/split_variants.py q16 q16nk q24 q33 q16 > gpurun_out/r04_quad_ring.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c2prof -o c2 -- python3 tools/c2_probe.py 20 > gpurun_out/r04_c2_probe.txt 2>&1

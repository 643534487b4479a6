# Training step with the residual folded into the forward panel GEMM (two-kernel schedule):
# training / out-grad parity tests, then the schedule probe (2 x 10 000 and 2 x 100 000).
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1
  local rc=$?
  echo "step $name rc=$rc"
  case $rc in 0) ;; *) echo "stopping after $name"; tail -30 "gpurun_out/r04_$name.log"; exit $rc;; esac
  return 0
}
step train_tests 600 python -u -m pytest tests/test_train.py tests/test_out_grad.py -m gpu -x -q --timeout 300 --timeout-method thread
step train_sched3 300 python -u tools/train_sched_probe.py 10
tail -2 gpurun_out/r04_train_tests.log
cat gpurun_out/r04_train_sched3.log | grep -v amdgpu.ids

# GPU suite on the 24-deep quad ring build, C5 A/B, training schedules with early HBM loads,
# then the bench line.
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1
  local rc=$?
  echo "step $name rc=$rc"
  case $rc in 124|134|137|139) echo "stopping after $name"; tail -20 "gpurun_out/r04_$name.log"; exit $rc;; esac
  return 0
}
step gpu_tests2 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step c5_ab 300 python -u tests/diag/c5_variants.py q16 q24k q24s22 q16 q24k q24s22 q16 q24k q24s22
step train_sched2 300 python -u tools/train_sched_probe.py 10
step bench2 600 python -u bench.py --steps 20 --warmup 5
tail -3 gpurun_out/r04_gpu_tests2.log

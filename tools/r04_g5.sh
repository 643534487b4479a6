# round-4 GPU pass: full GPU suite, training schedules, C5 ring-depth variants, C2 profile,
# bench line.  Stops at the first step that times out or crashes (GPU fault safety).
mkdir -p gpurun_out
step() {   # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1
  local rc=$?
  echo "step $name rc=$rc"
  case $rc in 124|134|137|139) echo "stopping after $name"; tail -20 "gpurun_out/r04_$name.log"; exit $rc;; esac
  return 0
}
step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step train_sched 300 python -u tools/train_sched_probe.py 10
step c5_variants 300 python -u tests/diag/c5_variants.py q16 q16nk q24 q33 q16
step c2_probe 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c2prof -o c2 -- python3 tools/c2_probe.py 20
step bench 600 python -u bench.py --steps 20 --warmup 5
tail -3 gpurun_out/r04_gpu_tests.log

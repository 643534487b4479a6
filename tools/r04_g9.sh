# Quad layers with the rotated-row ring reduction: quad/planner tests first, then the whole GPU
# suite and the bench line (C5 time in its extras).
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1
  local rc=$?
  echo "step $name rc=$rc"
  case $rc in 0) ;; *) echo "stopping after $name"; tail -30 "gpurun_out/r04_$name.log"; exit $rc;; esac
  return 0
}
step quad_tests 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "quad or plan or w2 or solo or handoff"
step gpu_tests3 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench3 600 python -u bench.py --steps 20 --warmup 5
tail -3 gpurun_out/r04_gpu_tests3.log
tail -1 gpurun_out/r04_bench3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: v for k, v in d['extras'].items() if k.startswith('c5_arm_plan_1024q_ms') or k=='c5_arm_plan_us_per_step'}, d['value'])" || true

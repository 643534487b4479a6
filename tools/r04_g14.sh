# Final-candidate build (pinned 16-deep quad ring, compact quad bias vectors, wide head row in
# LDS): whole GPU suite, then the bench line.
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1
  local rc=$?
  echo "step $name rc=$rc"
  case $rc in 0) ;; *) echo "stopping after $name"; tail -30 "gpurun_out/r04_$name.log"; exit $rc;; esac
  return 0
}
step gpu_tests5 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench5 600 python -u bench.py --steps 20 --warmup 5
tail -3 gpurun_out/r04_gpu_tests5.log
tail -1 gpurun_out/r04_bench5.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print(d['value'], d['roofline']['frac'], e['headline_1M_wave_tile_kernel_ms'], e['c5_arm_plan_1024q_ms'], e['gib_plan_q1_ms_per_step_auto'], e['train_step_2x10000_ms'])"

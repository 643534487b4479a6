# Quad kernels with the rotated-row ring reduction and pinned weight-ring loads (16 MFMA / 22
# SOLO): quad/planner parity tests, the whole GPU suite, C5 A/B against perf builds, bench line.
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1
  local rc=$?
  echo "step $name rc=$rc"
  case $rc in 0) ;; *) echo "stopping after $name"; tail -30 "gpurun_out/r04_$name.log"; exit $rc;; esac
  return 0
}
step quad_tests4 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "quad or plan or w2 or solo or handoff"
step gpu_tests4 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step c5_ab4 300 python -u tests/diag/c5_variants.py q16p q24 q24nkp q22nkp q16p q24 q24nkp q22nkp
step bench4 600 python -u bench.py --steps 20 --warmup 5
tail -3 gpurun_out/r04_gpu_tests4.log
cat gpurun_out/r04_c5_ab4.log

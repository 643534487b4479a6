# Weight-gradient kernel check on one GPU: the whole -m gpu suite, the GEMM probe with the
# wgrad kernel (default) and the LDS-tiled split-K kernel (PNTF_GEMM_WGRAD=0), the training
# step per kernel, then the headline profiles and the default bench line (tools/r03_full.sh).
set -e
export PYTHONUNBUFFERED=1
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests \
  > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
for m in 1 0; do
  PNTF_GEMM_WGRAD=$m timeout -k 10 300 python -u tools/gemm_probe.py 20000 mfma > "$OUT/gemm_probe_wgrad$m.json"
  echo "wgrad $m"; python3 -c "
import json; d = json.load(open('$OUT/gemm_probe_wgrad$m.json'))
print({t: {k: v for k, v in r.items() if 'bwdw' in k} for t, r in d.items()})"
done
bash tools/prof_train.sh > "$OUT/train_prof.txt" 2>&1
cat "$OUT/train_prof.txt"
bash tools/profile_round.sh
echo PROFILED
timeout -k 10 600 python3 bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail -20 "$OUT/bench_default.err"; exit 1; }
cat "$OUT/bench_default.json"

# Fused Linear + act_laplace check on one GPU: the training tests, the training step per
# kernel, and the step time with the fused kernel (default) and the two-kernel path
# (PNTF_TT_FUSED=0).
set -e
export PYTHONUNBUFFERED=1
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_train.py \
  > "$OUT/train_tests.log" 2>&1 || { tail -40 "$OUT/train_tests.log"; exit 1; }
tail -1 "$OUT/train_tests.log"
bash tools/prof_train.sh > "$OUT/train_prof.txt" 2>&1
cat "$OUT/train_prof.txt"
for m in 1 0; do
  PNTF_TT_FUSED=$m timeout -k 10 300 python3 bench.py --train-only > "$OUT/train_only_$m.json" 2>&1
  echo "fused $m"; tail -c 600 "$OUT/train_only_$m.json"; echo
done

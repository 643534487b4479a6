# Iteration pass: the -m gpu tests matching $1 (all when empty), C5 timings (AUTO = hand-off,
# QUAD_TILE = without) and the training step timings + per-kernel profile.
set -e
export PYTHONUNBUFFERED=1
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
K=${1:-}
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests \
  ${K:+-k "$K"} > "$OUT/iter_tests.log" 2>&1 || { tail -40 "$OUT/iter_tests.log"; exit 1; }
tail -2 "$OUT/iter_tests.log"
timeout -k 10 120 python3 tools/c5_probe.py 5 auto
timeout -k 10 120 python3 tools/c5_probe.py 5 quad_tile
timeout -k 10 300 python3 bench.py --train-only
bash tools/prof_train.sh > "$OUT/train_prof.txt" 2>&1
cat "$OUT/train_prof.txt"

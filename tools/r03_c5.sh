# C5 planner iteration: planner tests, then C5 timings (AUTO = hand-off, QUAD_TILE = without)
set -e
export PYTHONUNBUFFERED=1
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests \
  -k "planner or plan or solo or c5 or tail" > "$OUT/c5_tests.log" 2>&1 || { tail -40 "$OUT/c5_tests.log"; exit 1; }
tail -3 "$OUT/c5_tests.log"
timeout -k 10 120 python3 tools/c5_probe.py 5 auto
timeout -k 10 120 python3 tools/c5_probe.py 5 quad_tile

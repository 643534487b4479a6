# Round-3 checkpoint on one GPU: the whole -m gpu suite, the training step per kernel, the C5
# planner (step distribution, stream roofline), the stream probe, then the default bench line.
# The headline PMC passes (tools/profile_round.sh) run only when $1 = prof.
set -e
export PYTHONUNBUFFERED=1
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests \
  > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
bash tools/prof_train.sh > "$OUT/train_prof.txt" 2>&1
cat "$OUT/train_prof.txt"
timeout -k 10 120 python3 tools/c5_probe.py 5 auto > "$OUT/c5.txt" 2>&1
cat "$OUT/c5.txt"
timeout -k 10 120 tests/diag/stream_probe > "$OUT/stream_probe.txt" 2>&1
cat "$OUT/stream_probe.txt"
if [ "${1:-}" = prof ]; then bash tools/profile_round.sh; echo PROFILED; fi
timeout -k 10 600 python3 bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail -20 "$OUT/bench_default.err"; exit 1; }
cat "$OUT/bench_default.json"

# Round-4 closing pass after the training-epilogue change (gemm / train units and pntf/train.py
# only; the wide and quad units, whose PMC summaries are stamped, are unchanged): the -m gpu
# suite, training per-kernel stats, the default bench line, smoke().
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > "$OUT/r04_final3_gpu_tests.log" 2>&1 || { tail -40 "$OUT/r04_final3_gpu_tests.log"; exit 1; }
tail -2 "$OUT/r04_final3_gpu_tests.log"
bash tools/prof_train.sh > "$OUT/train_prof3.txt" 2>&1
head -8 "$OUT/train_prof3.txt"
timeout -k 10 600 python3 bench.py > "$OUT/bench_default3.json" 2> "$OUT/bench_default3.err" || { tail -20 "$OUT/bench_default3.err"; exit 1; }
cat "$OUT/bench_default3.json"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tests/diag/pair32_probe > gpurun_out/r04_pair32.txt 2>&1 || echo "pair probe rc=$?"
timeout -k 10 400 python -u tests/diag/perf_variants.py wbase wnoload whot wnost wnone wcheap wcheapnone wbase > gpurun_out/r04_wide_ablation.txt 2>&1

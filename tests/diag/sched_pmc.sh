#!/bin/bash
# PMC comparison of the 16-pair and 32-pair τ+∇τ kernels (tests/diag/sched_pmc.py).
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
cd /tmp && export TMPDIR=/tmp
i=0
for C in "$@"; do
  OUT=$R/gpurun_out/spmc$i; rm -rf "$OUT"; mkdir -p "$OUT"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d "$OUT" -o run --output-format csv -- \
    python3 "$R/tests/diag/sched_pmc.py" > "$OUT/log.txt" 2>&1
  python3 "$R/tests/diag/sched_pmc.py" --parse "$OUT"
  i=$((i+1))
done

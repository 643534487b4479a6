#!/bin/bash
# PMC comparison of perf variants (tests/diag/libperf_<name>.so): one rocprofv3 pass with
# wave-cycle, wait, MFMA-busy and clock counters over perf_variants.py; summarised per variant
# by pmc_parse.py (dispatch order: the shipped kernel once, then 6 launches per variant).
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
OUT=$R/gpurun_out/pmcv
rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
COUNTERS=${COUNTERS:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE}
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $COUNTERS -d "$OUT" -o run --output-format csv -- \
  python3 "$R/tests/diag/perf_variants.py" "$@" > "$OUT/log.txt" 2>&1
python3 "$R/tests/diag/pmc_parse.py" "$OUT" "$@"

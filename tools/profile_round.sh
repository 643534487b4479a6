#!/bin/bash
# Profile the headline τ+∇τ kernel on the GPU box (run through gpurun from the repo root):
# kernel-trace --stats, then separate PMC passes (MI355X_MICROARCH.md: FETCH_SIZE and
# WRITE_SIZE cannot share a pass), then the stall counters.  Outputs land in gpurun_out/;
# tools/prof_summary.py turns them into the committed profiles/ files.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --no-cpu --no-extra --roofline-launches 1"
run() {  # run <dir> <seconds> <rocprofv3 args...>
  local d=$1 t=$2; shift 2
  timeout -k 10 "$t" rocprofv3 "$@" -d "$OUT/$d" -o run --output-format csv -- \
    python3 $BENCH --steps ${STEPS:-3} --warmup 1 > "$OUT/$d.log" 2>&1
}
# the stats pass times 20 steps, so the one cold first launch weighs 1/27 of the mean
STEPS=20 run prof_stats 300 --kernel-trace --stats
run pmc_fetch 300 --pmc FETCH_SIZE
run pmc_write 300 --pmc WRITE_SIZE
run pmc_mfma 300 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1
run pmc_stall 300 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY

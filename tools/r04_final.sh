# Round-4 final pass on one GPU (pinned 16-deep quad ring, wide head row + env-B table in LDS): the -m gpu suite, the C5
# planner (stats + PMC passes), the stream probes, the Q1 planner step, the headline profile
# (tools/profile_round.sh: stats + FETCH/WRITE/MFMA/stall PMC), then the default bench line.
# Outputs in gpurun_out/; tools/prof_summary.py and tools/c5_pmc_summary.py turn them into
# profiles/.  Each GPU step has its own time limit; any failure ends the script.
set -e
export PYTHONUNBUFFERED=1
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests \
  > "$OUT/r04_final_gpu_tests.log" 2>&1 || { tail -40 "$OUT/r04_final_gpu_tests.log"; exit 1; }
tail -2 "$OUT/r04_final_gpu_tests.log"
timeout -k 10 120 python3 tools/q1_probe.py > "$OUT/q1.txt" 2>&1
cd /tmp && export TMPDIR=/tmp
C5="$R/tools/c5_probe.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/c5_stats" -o run --output-format csv -- \
  python3 $C5 5 > "$OUT/c5_stats.log" 2>&1
tail -1 "$OUT/c5_stats.log"
pmc() {  # pmc <tag> <counters...>
  local t=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/c5_pmc_$t" -o run --output-format csv -- \
    python3 $C5 2 > "$OUT/c5_pmc_$t.log" 2>&1
}
pmc sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS
pmc tcc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE
pmc fetch FETCH_SIZE
pmc lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_SMEM
echo C5_PMC_DONE
cd "$R"
bash tools/profile_round.sh
echo PROFILED
bash tools/prof_train.sh > "$OUT/train_prof.txt" 2>&1
echo TRAIN_PROFILED
# stamp the headline PMC summary here, so the bench line below reports roofline.traffic
python3 tools/prof_summary.py --tag r04 --pairs 1048576 > "$OUT/prof_summary.txt" 2>&1
cp profiles/pmc_tau_grad.json "$OUT/pmc_tau_grad.json"
timeout -k 10 600 python3 bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail -20 "$OUT/bench_default.err"; exit 1; }
cat "$OUT/bench_default.json"

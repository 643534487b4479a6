#!/bin/bash
# One parameterised GPU pass (run through gpurun from the repo root); every profiles/r05_*
# file comes from one of its steps.
#
#   tools/gpu_pass.sh <tag> <step>...
#
# steps (each under its own time limit, chained: the first failure ends the pass):
#   tests[=<pytest args>]  the -m gpu suite (default: all of tests/), log <tag>_gpu_tests.log;
#                          alltests[=...] runs past failures (reports them, goes on)
#   bench                  the default bench.py line -> <tag>_bench.json
#   head                   headline kernel: rocprofv3 stats over 20 steps + FETCH/WRITE/MFMA/
#                          stall PMC passes (tools/profile_round.sh) -> <tag>_prof/
#   c5                     C5 planner: kernel trace + stats, then the SQ / TCC / LDS PMC passes
#   q1                     batch-1 Gibson planner step probe (tools/q1_probe.py)
#   train                  training-step kernel trace at 2 x 10 000 pairs (tools/prof_train.sh)
#   py=<tool.py args>      a probe script (tools/*.py), output <tag>_<tool>.txt
#   trace=<tool.py args>   the same under rocprofv3 --kernel-trace --stats, plus the idle-gap
#                          summary of tools/trace_gaps.py
#   pmc=<name>:<c1,c2,..>:<tool.py args>  one PMC pass (counters only) over a probe script
#   smoke                  __graft_entry__.smoke()
# Outputs land in gpurun_out/<tag>_*; tools/prof_summary.py / c5_pmc_summary.py turn them
# into profiles/.
set -e
export PYTHONUNBUFFERED=1
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
TAG=$1; shift
cd "$R"
for step in "$@"; do
  echo "== $step $(date +%T)"
  case "$step" in
    tests*|alltests*)
      # tests: stop at the first failure and end the pass; alltests: run every test, report
      # the failures and go on (kernel faults still end the pass: their exit status is not 1)
      x=-x; [ "${step#all}" != "$step" ] && x=; s0=${step#all}
      args=${s0#tests}; args=${args#=}; [ -z "$args" ] && args=tests
      rc=0
      timeout -k 10 1200 python -u -m pytest $x -v -s --timeout 300 --timeout-method thread \
        -m gpu $args > "$OUT/${TAG}_gpu_tests.log" 2>&1 || rc=$?
      tail -3 "$OUT/${TAG}_gpu_tests.log"
      if [ $rc -ne 0 ]; then
        grep -E "^FAILED|^ERROR" "$OUT/${TAG}_gpu_tests.log" | head -40
        [ -n "$x" ] || [ $rc -ne 1 ] && exit 1
      fi ;;
    bench)
      timeout -k 10 900 python3 bench.py > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err" \
        || { tail -30 "$OUT/${TAG}_bench.err"; exit 1; }
      cat "$OUT/${TAG}_bench.json" ;;
    head)
      bash tools/profile_round.sh
      for d in prof_stats pmc_fetch pmc_write pmc_mfma pmc_stall; do
        rm -rf "$OUT/${TAG}_$d"; mv "$OUT/$d" "$OUT/${TAG}_$d"; mv "$OUT/$d.log" "$OUT/${TAG}_$d.log"
      done ;;
    c5)
      ( cd /tmp && export TMPDIR=/tmp
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_c5_stats" -o run \
          --output-format csv -- python3 "$R/tools/c5_probe.py" 10 > "$OUT/${TAG}_c5_stats.log" 2>&1
        tail -1 "$OUT/${TAG}_c5_stats.log"
        pmc() { local t=$1; shift
          timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/${TAG}_c5_pmc_$t" -o run \
            --output-format csv -- python3 "$R/tools/c5_probe.py" 2 > "$OUT/${TAG}_c5_pmc_$t.log" 2>&1; }
        pmc sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS
        pmc tcc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE
        pmc fetch FETCH_SIZE
        pmc lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_SMEM
      ) ;;
    q1)
      timeout -k 10 120 python3 tools/q1_probe.py > "$OUT/${TAG}_q1.txt" 2>&1; tail -3 "$OUT/${TAG}_q1.txt" ;;
    train)
      bash tools/prof_train.sh > "$OUT/${TAG}_train_prof.txt" 2>&1
      rm -rf "$OUT/${TAG}_prof_train"; mv "$OUT/prof_train" "$OUT/${TAG}_prof_train"
      cat "$OUT/${TAG}_train_prof.txt" ;;
    py=*)       # py=<tool.py args...>: a probe script, output <tag>_<tool>.txt
      a=${step#py=}; nm=$(basename ${a%% *} .py)
      timeout -k 10 600 python3 $a > "$OUT/${TAG}_$nm.txt" 2>&1 || { tail -30 "$OUT/${TAG}_$nm.txt"; exit 1; }
      tail -5 "$OUT/${TAG}_$nm.txt" ;;
    trace=*)    # trace=<tool.py args...>: kernel trace (no counters) + idle-gap summary
      a=${step#trace=}; nm=$(basename ${a%% *} .py)
      ( cd /tmp && export TMPDIR=/tmp
        timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_trace_$nm" -o run \
          --output-format csv -- python3 $R/$a > "$OUT/${TAG}_trace_$nm.log" 2>&1 )
      f=$(find "$OUT/${TAG}_trace_$nm" -name "*kernel_trace.csv" | head -1)
      python3 tools/trace_gaps.py "$f" | tee "$OUT/${TAG}_trace_$nm.gaps" ;;
    pmc=*)      # pmc=<name>:<counter,...>:<tool.py args...>: one counter pass over a probe
      a=${step#pmc=}; nm=${a%%:*}; a=${a#*:}; ctr=${a%%:*}; a=${a#*:}
      ( cd /tmp && export TMPDIR=/tmp
        timeout -s KILL 180 rocprofv3 --pmc ${ctr//,/ } -d "$OUT/${TAG}_pmc_$nm" -o run \
          --output-format csv -- python3 $R/$a > "$OUT/${TAG}_pmc_$nm.log" 2>&1 ) \
        || { tail -20 "$OUT/${TAG}_pmc_$nm.log"; exit 1; }
      tail -2 "$OUT/${TAG}_pmc_$nm.log" ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"

#!/bin/bash
set -e
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() { local d=$1; shift; timeout -k 10 200 rocprofv3 "$@" -d "$OUT/$d" -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-extra --roofline-launches 1 --steps 3 --warmup 1 > "$OUT/$d.log" 2>&1; }
run pmc_icache --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH
run pmc_tcc --pmc TCC_HIT_sum TCC_MISS_sum
run pmc_tcp --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum

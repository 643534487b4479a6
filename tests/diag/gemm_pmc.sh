#!/bin/bash
# PMC pass over the GEMM variant harness (diagnostics).
set -e
R=$(pwd)
OUT=$R/gpurun_out/gemm_pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY -d $OUT -o run --output-format csv -- python3 $R/tests/diag/gemm_variants.py m128 > $OUT/log 2>&1
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('/root/repo/gpurun_out/gemm_pmc/**/*counter_collection.csv', recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    n = r['Kernel_Name']
    if 'gemm_kernel' not in n: continue
    agg[n[:60]][r['Counter_Name']] += float(r['Counter_Value'])
for n, d in agg.items():
    print(n, {k: '%.3g' % v for k, v in d.items()})
PY

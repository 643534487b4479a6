#!/bin/bash
# PMC passes over the training GEMM shapes (tools/gemm_probe.py one-shape mode): wave-cycle
# split, MFMA busy and LDS counters of the panel kernels, summarised per kernel.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/panel_pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/a -o run --output-format csv -- python3 $R/tools/gemm_probe.py 20000 one > $OUT/a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU -d $OUT/b -o run --output-format csv -- python3 $R/tools/gemm_probe.py 20000 one > $OUT/b.log 2>&1
python3 - <<'PY'
import csv, glob, collections
for p in ('a', 'b'):
    f = glob.glob('/root/repo/gpurun_out/panel_pmc/%s/**/*counter_collection.csv' % p, recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name']
        if 'panel' not in n: continue
        agg[n[:64]][r['Counter_Name']] += float(r['Counter_Value'])
    for n, d in agg.items():
        print(p, n, {k: '%.4g' % v for k, v in d.items()})
PY

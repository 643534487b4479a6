# Weight-gradient GEMM evidence on one GPU: the GEMM parity tests, then rocprofv3 kernel stats
# of the GEMM probe with the wgrad kernel (default) and the LDS-tiled split-K kernel
# (PNTF_GEMM_WGRAD=0; 2 = the two-buffer burst variant, PNTF_WGRAD_RING=2), and the HBM fetch / MFMA-busy PMC passes of the wgrad kernel.
set -e
export PYTHONUNBUFFERED=1
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_train.py \
  > "$OUT/gemm_tests.log" 2>&1 || { tail -40 "$OUT/gemm_tests.log"; exit 1; }
tail -1 "$OUT/gemm_tests.log"
cd /tmp && export TMPDIR=/tmp
for m in 1 2 0; do
  PNTF_WGRAD_RING=$m PNTF_GEMM_WGRAD=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/wgrad_prof$m" -o p --output-format csv -- \
    python3 "$R/tools/gemm_probe.py" 20000 mfma > "$OUT/wgrad_probe$m.json" 2> "$OUT/wgrad_probe$m.err"
  echo "wgrad $m"; python3 -c "
import json; d = json.load(open('$OUT/wgrad_probe$m.json'))
print({t: {k: v for k, v in r.items() if 'bwdw' in k} for t, r in d.items()})"
  f=$(find "$OUT/wgrad_prof$m" -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if any(k in r['Name'] for k in ('wgrad', 'gemm_kernel', 'reduce')):
        print('%8.1f us %5s  %s' % (float(r['AverageNs']) / 1e3, r['Calls'], r['Name'][:70]))"
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex wgrad -d "$OUT/wgrad_pmc_fetch" -o p --output-format csv -- \
  python3 "$R/tools/gemm_probe.py" 20000 mfma > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES --kernel-include-regex wgrad -d "$OUT/wgrad_pmc_mfma" -o p --output-format csv -- \
  python3 "$R/tools/gemm_probe.py" 20000 mfma > /dev/null 2>&1
echo PMC done

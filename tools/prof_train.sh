# rocprofv3 kernel stats of the training step (bench.py --train-only: 2x10000 and 2x100000).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_train
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o train --output-format csv -- python3 bench.py --train-only > gpurun_out/prof_train/out.json 2> gpurun_out/prof_train/err.log
f=$(find gpurun_out/prof_train -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:14]:
    print('%6.1f%% %8.2f ms %5s  %s'%(100*float(r['TotalDurationNs'])/tot,float(r['TotalDurationNs'])/1e6,r['Calls'],r['Name'][:90]))
"

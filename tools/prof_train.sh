# rocprofv3 kernel stats of the training step at the reference batch (tools/train_profile.py:
# 2 envs x 10 000 pairs, 1 warm + 5 timed steps), summarised per kernel.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/prof_train
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train -o train --output-format csv -- python3 $R/tools/train_profile.py 10000 > $R/gpurun_out/prof_train/out.json 2> $R/gpurun_out/prof_train/err.log
f=$(find $R/gpurun_out/prof_train -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
tot=sum(float(r['TotalDurationNs']) for r in rows)
print('total %.2f ms over 6 steps'%(tot/1e6))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:12]:
    print('%6.1f%% %8.2f ms %5s  %s'%(100*float(r['TotalDurationNs'])/tot,float(r['TotalDurationNs'])/1e6,r['Calls'],r['Name'][:90]))
"

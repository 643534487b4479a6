# rocprofv3 kernel stats over every bench config (headline + extras: split / quad planners,
# residual, training GEMMs, mesh distance); run through gpurun from the repo root.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_all" -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu --roofline-launches 1 --steps 3 --warmup 1 > "$OUT/prof_all.log" 2>&1

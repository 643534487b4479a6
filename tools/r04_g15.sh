# Wide kernel: env-B table in LDS (wbl) vs global B reads (wbase), 1M pairs, against the shipped kernel.
mkdir -p gpurun_out
timeout -k 10 400 python -u tests/diag/perf_variants.py wbase wbl wbase wbl wbase wbl > gpurun_out/r04_wide_bl.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04_wide_bl.log; exit $rc

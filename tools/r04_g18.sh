# Wide kernel ablation: the softplus/sigma scaling multiply dropped (wrong results, timing only).
mkdir -p gpurun_out
timeout -k 10 400 python -u tests/diag/perf_variants.py wbl wnoscale wbl wnoscale wbl wnoscale > gpurun_out/r04_wide_noscale.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04_wide_noscale.log | grep -v "bad pairs"; exit $rc

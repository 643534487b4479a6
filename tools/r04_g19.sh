# kappa-scaled wide activations: same-box A/B against the previous wide code (perf build of the
# last commit's headers; it reads the new scaled blob, so its results are wrong: timing only),
# then the full round-4 final pass (GPU suite, profiles, PMC stamp, bench line).
mkdir -p gpurun_out
timeout -k 10 400 python -u tests/diag/perf_variants.py wold wk wold wk wold wk > gpurun_out/r04_wide_kappa.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04_wide_kappa.log | grep -v "bad pairs"; [ $rc -eq 0 ] || exit $rc
bash tools/r04_final.sh

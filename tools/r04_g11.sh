# C5 perf-variant harness check: per-variant step counts and path differences vs the shipped plan.
mkdir -p gpurun_out
timeout -k 10 300 python -u tests/diag/c5_variants.py qnopin qpin16s22 qpin24nk > gpurun_out/r04_c5_pin2.log 2>&1
rc=$?; cat gpurun_out/r04_c5_pin2.log; exit $rc

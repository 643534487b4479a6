# C5 A/B on the pinned 16-deep ring: compact bias vectors (a16p), static priority for waves 4-7,
# SOLO ring 16, ring 12, one accumulator chain.
mkdir -p gpurun_out
timeout -k 10 400 python -u tests/diag/c5_variants.py a16p a16prio a16s16 a12p a16c1 a16p a16prio a16s16 a12p a16c1 > gpurun_out/r04_c5_ab5.log 2>&1
rc=$?; cat gpurun_out/r04_c5_ab5.log; exit $rc

# C5 A/B: quad weight-ring loads pinned in program order (sched_barrier) at several ring depths,
# with / without the B operands kept in registers, against the unpinned 24/22 build; then wide
# kernel ablations of the env-B and head-row loads.
mkdir -p gpurun_out
timeout -k 10 400 python -u tests/diag/c5_variants.py qnopin qpin16s22 qpin22nk qpin24nk qnopin qpin16s22 qpin22nk qpin24nk > gpurun_out/r04_c5_pin.log 2>&1
rc=$?; cat gpurun_out/r04_c5_pin.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tests/diag/perf_variants.py wbase wnohw wnoboth wnobw wbase wnohw wnoboth wnobw > gpurun_out/r04_wide_bw.log 2>&1
rc=$?; cat gpurun_out/r04_wide_bw.log; exit $rc

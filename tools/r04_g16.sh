# Quad tau+grad step ablations on the pinned 16-deep ring (field_quad_kernel<3,1>, 1 / 4 / 256
# tiles): base, unpinned, no barriers, no weight loads, no LDS reads (wrong results, timing only).
mkdir -p gpurun_out
timeout -k 10 300 python -u tests/diag/split_variants.py f16p f16u fnobar fnoload fnolds f16p f16u > gpurun_out/r04_quad_abl.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04_quad_abl.log; exit $rc

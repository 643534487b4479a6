#!/bin/bash
# Build variants of csrc/pntf_gemm.hip as standalone libraries (with pntf_train.hip, whose act
# kernels pntf_tt_linear_act calls): name=flags pairs.
set -e
cd "$(dirname "$0")/../.."
for v in "$@"; do
  name=${v%%=*}; flags=${v#*=}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -Iinclude \
    -Xclang -target-feature -Xclang -packed-fp32-ops $flags p-ntfields_amd/csrc/pntf_gemm.hip p-ntfields_amd/csrc/pntf_train.hip \
    -o tests/diag/libgemm_$name.so &
done
wait

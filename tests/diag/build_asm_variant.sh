#!/bin/bash
# Build perf variants of the wide kernel with their assembly kept (tests/diag/asmv_<name>/),
# for register / spill inspection:  build_asm_variant.sh name="flags" ...
# (the .so is copied to tests/diag/libperf_<name>.so for perf_variants.py)
cd "$(dirname "$0")/../.."
for v in "$@"; do
  name=${v%%=*}; flags=${v#*=}
  d=tests/diag/asmv_$name; rm -rf $d; mkdir -p $d
  ( /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -Iinclude \
      -Ip-ntfields_amd/csrc -Xclang -target-feature -Xclang -packed-fp32-ops -save-temps=obj $flags \
      tests/diag/perf_variant.hip -o $d/libperf_$name.so -Rpass-analysis=kernel-resource-usage \
      2> $d/remarks.txt && cp $d/libperf_$name.so tests/diag/
    echo "$name: $(grep -A8 'wide_field_kernel' $d/remarks.txt | grep -oE '(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|VGPRs Spill): [0-9]+' | tr '\n' ' ')" ) &
done
wait

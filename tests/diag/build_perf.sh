#!/bin/bash
# Build perf variants of the τ+∇τ kernel: name=flags pairs; prints each one's resource usage.
# A +pk token in the flags builds with packed-fp32 VALU codegen (v_pk_{mul,add,fma}_f32) enabled.
set -e
cd "$(dirname "$0")/../.."
build() {
  local name=$1; shift
  local pk="-Xclang -target-feature -Xclang -packed-fp32-ops" a=()
  for f in "$@"; do if [ "$f" = "+pk" ]; then pk=; else a+=("$f"); fi; done
  set -- "${a[@]}"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -Iinclude \
    -Ip-ntfields_amd/csrc $pk "$@" tests/diag/perf_variant.hip -o tests/diag/libperf_$name.so \
    -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "VGPRs:|AGPRs|Spill" | tr '\n' ' ' \
    | sed "s/^/$name: /"; echo
}
for v in "$@"; do
  name=${v%%=*}; flags=${v#*=}
  build $name $flags &
done
wait

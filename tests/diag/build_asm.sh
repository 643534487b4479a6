#!/bin/bash
# Build code objects (tests/diag/hsaco_<name>.hsaco) of perf_variant.hip's τ+∇τ kernel from
# patched assembly: build_asm.sh "<name>=<policy>[:states]|<hipcc flags>" ...
set -e
cd "$(dirname "$0")/../.."
LLVM=/opt/rocm/lib/llvm/bin
for v in "$@"; do
  name=${v%%=*}; rest=${v#*=}; pol=${rest%%|*}; flags=${rest#*|}
  policy=${pol%%:*}; states=24; [ "$pol" != "$policy" ] && states=${pol#*:}
  tmp=$(mktemp -d)
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --offload-device-only -S -Iinclude \
    -Ip-ntfields_amd/csrc $flags tests/diag/perf_variant.hip -o $tmp/k.s 2>/dev/null
  python3 tests/diag/asm_patch.py $policy $tmp/k.s $tmp/p.s $states
  $LLVM/clang -target amdgcn-amd-amdhsa -mcpu=gfx950 -c $tmp/p.s -o $tmp/p.o
  $LLVM/ld.lld -shared $tmp/p.o -o tests/diag/hsaco_$name.hsaco
  rm -rf $tmp
done

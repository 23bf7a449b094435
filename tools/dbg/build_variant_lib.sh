#!/bin/bash
# Probe recipe (not product code): libbpsr from the working tree's sources as
# they stand, into tools/dbg/<name>/libbpsr.so (extra compiler flags after the
# name), for same-box A/Bs against prophet_amd/libbpsr.so: on the GPU box copy
# it over prophet_amd/libbpsr.so between runs.
#   tools/dbg/build_variant_lib.sh <name> [-DFLAG ...]
set -euo pipefail
cd "$(dirname "$0")/../.."
name=$1; shift
out=tools/dbg/$name
mkdir -p "$out/obj"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fvisibility=hidden \
   -fvisibility-inlines-hidden -fno-gpu-rdc -mllvm -amdgpu-atomic-optimizer-strategy=None \
   -Wno-unused-function -Iinclude -Iprophet_amd/csrc $*"
objs=""
for src in prophet_amd/csrc/*.hip prophet_amd/csrc/*.cpp; do
  o="$out/obj/$(basename "$src").o"
  /opt/rocm/bin/hipcc $F -c "$src" -o "$o" &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 \
  -Wl,--version-script=prophet_amd/csrc/bpsr.lds -o "$out/libbpsr.so" $objs -ldl
rm -rf "$out/obj"
echo "$out/libbpsr.so"

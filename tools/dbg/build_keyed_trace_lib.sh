#!/bin/bash
# Probe recipe (not product code), round 6: libbpsr with -DBPSR_KEYED_TRACE
# (the keyed consumer's per-tile wall-clock stamps, dumped at queue destroy to
# $BPSR_KEYED_TRACE_OUT), built beside the product into tools/dbg/ktrace/.
# On the GPU box (a scratch copy of the tree) copy it over
# prophet_amd/libbpsr.so before running a driver; tools/dbg/keyed_trace_report.py
# reads the dump.
set -euo pipefail
cd "$(dirname "$0")/../.."
out=tools/dbg/ktrace
mkdir -p "$out/obj"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fvisibility=hidden \
   -fvisibility-inlines-hidden -fno-gpu-rdc -mllvm -amdgpu-atomic-optimizer-strategy=None \
   -Wno-unused-function -Iinclude -Iprophet_amd/csrc -DBPSR_KEYED_TRACE"
objs=""
for src in prophet_amd/csrc/*.hip prophet_amd/csrc/*.cpp; do
  o="$out/obj/$(basename "$src").o"
  /opt/rocm/bin/hipcc $F -c "$src" -o "$o" &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 \
  -Wl,--version-script=prophet_amd/csrc/bpsr.lds -o "$out/libbpsr.so" $objs -ldl
echo "$out/libbpsr.so"

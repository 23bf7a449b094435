#!/bin/bash
# Probe recipe (not product code), round 6: libbpsr with bpsr_api.cpp as of a
# given commit (default: round 5's last, 39ef088) and every other object of the
# current build, for the A/B of tests/blockq_shared_hwq_case.py
# (profiles/r06s04_shared_hwq_ab.txt).  Output: tools/dbg/old_api/libbpsr.so.
#   make -C prophet_amd/csrc && tools/dbg/build_old_api_lib.sh [commit]
set -euo pipefail
cd "$(dirname "$0")/../.."
rev=${1:-39ef088}
out=tools/dbg/old_api
mkdir -p "$out"
git show "$rev:prophet_amd/csrc/bpsr_api.cpp" > prophet_amd/csrc/_old_api.cpp
trap 'rm -f prophet_amd/csrc/_old_api.cpp' EXIT
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fvisibility=hidden \
   -fvisibility-inlines-hidden -fno-gpu-rdc -mllvm -amdgpu-atomic-optimizer-strategy=None \
   -Wno-unused-function -Iinclude -Iprophet_amd/csrc"
/opt/rocm/bin/hipcc $F -c prophet_amd/csrc/_old_api.cpp -o "$out/api.o"
objs=$(ls prophet_amd/csrc/build/*.o | grep -v 'bpsr_api.cpp.o')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 \
  -Wl,--version-script=prophet_amd/csrc/bpsr.lds -o "$out/libbpsr.so" $objs "$out/api.o" -ldl
rm -f "$out/api.o"
echo "$out/libbpsr.so"

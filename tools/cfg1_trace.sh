#!/bin/bash
# rocprofv3 kernel + memory-copy traces of the cfg1 pull-view variants (blocking vs non-blocking pushes)
set -u
OUT=gpurun_out/r01s48
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/sync -o t -- python tools/cfg1_trace.py > $OUT/sync.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/async -o t -- python tools/cfg1_trace.py async > $OUT/async.log 2>&1

#!/bin/bash
# block-queue parity tests, then cfg3 block-queue variants plain and under a rocprofv3 kernel trace
set -u
OUT=gpurun_out/${TAG:-r01_bq}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_blockq_gpu.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/blockq.log 2>&1 &&
timeout -k 10 300 python tools/bench_configs.py --only cfg3 > $OUT/cfg3_plain.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o cfg3 -- python tools/bench_configs.py --only cfg3 --variants blockq > $OUT/cfg3.log 2>&1

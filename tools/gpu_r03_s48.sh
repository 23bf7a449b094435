export TMPDIR=/tmp; mkdir -p gpurun_out/r03s48
OUT=gpurun_out/r03s48
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -k "record_prefetch or batched or plan" -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; exit $rc

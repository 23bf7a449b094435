export TMPDIR=/tmp; mkdir -p gpurun_out/r03s61
OUT=gpurun_out/r03s61
timeout -k 10 600 python -u -m pytest tests/test_bench_gpu.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -6 $OUT/tests.log; exit $rc

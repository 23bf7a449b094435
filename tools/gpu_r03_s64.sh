export TMPDIR=/tmp; mkdir -p gpurun_out/r03s64
OUT=gpurun_out/r03s64
timeout -k 10 900 python -u -m pytest tests/test_server_gpu.py tests/test_server_group_gpu.py tests/test_native_gpu.py tests/test_pipeline_gpu.py tests/test_knownanswer_gpu.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; grep -c PASSED $OUT/tests.log; grep -E "FAILED|ERROR|blocking_device_calls" $OUT/tests.log | head; tail -2 $OUT/tests.log; exit $rc

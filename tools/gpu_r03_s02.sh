export TMPDIR=/tmp; mkdir -p gpurun_out/r03s02
timeout -k 10 600 python -u -m pytest tests/test_server_group_gpu.py tests/test_server_gpu.py tests/test_blockq_gpu.py tests/test_pushloop_gpu.py -x -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r03s02/server.log 2>&1; rc=$?; tail -30 gpurun_out/r03s02/server.log; exit $rc

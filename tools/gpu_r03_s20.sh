export TMPDIR=/tmp; mkdir -p gpurun_out/r03s20
for v in 1 6 4; do
  timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 4 $v >> gpurun_out/r03s20/srv.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_server_gpu.py tests/test_server_group_gpu.py tests/test_native_gpu.py tests/test_pushpull_gpu.py -m gpu -x -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r03s20/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03s20/tests.log; exit $rc

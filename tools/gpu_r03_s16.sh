export TMPDIR=/tmp; mkdir -p gpurun_out/r03s16
for v in 4 0 2 5; do
  timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 4 $v >> gpurun_out/r03s16/srv.log 2>&1 || exit $?
done
BPSR_SERVER_INFLIGHT=1 timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 4 4 >> gpurun_out/r03s16/srv_if1.log 2>&1 || exit $?
BPSR_SERVER_INFLIGHT=4 timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 4 4 >> gpurun_out/r03s16/srv_if4.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_server_gpu.py tests/test_server_group_gpu.py tests/test_native_gpu.py -m gpu -x -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r03s16/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03s16/tests.log; exit $rc

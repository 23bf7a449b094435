export TMPDIR=/tmp; mkdir -p gpurun_out/r03s14
timeout -k 10 600 python -u -m pytest tests/test_server_gpu.py tests/test_server_group_gpu.py tests/test_pushloop_gpu.py -m gpu -x -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r03s14/tests.log 2>&1; rc=$?; tail -5 gpurun_out/r03s14/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 4 > gpurun_out/r03s14/srv.log 2>&1 || exit $?
BPSR_SERVER_COMBINE=0 timeout -k 10 300 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 4 > gpurun_out/r03s14/srv_nocomb.log 2>&1 || exit $?
timeout -k 10 300 tools/cfg3_native tools/cfg3_resnet50_table.txt 200 7 tools/cfg3_resnet50_tasks.txt > gpurun_out/r03s14/cfg3.log 2>&1
exit $rc

export TMPDIR=/tmp; mkdir -p gpurun_out/r03s25
for v in 4 6 8 2; do
  timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 4 $v >> gpurun_out/r03s25/srv.log 2>&1 || exit $?
done
for v in 4 6; do
  timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 1 $v >> gpurun_out/r03s25/srv_1lane.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_server_gpu.py tests/test_server_group_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r03s25/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03s25/tests.log; exit $rc

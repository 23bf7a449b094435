export TMPDIR=/tmp; mkdir -p gpurun_out/r03s19
for v in 6 4 2; do
  timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 4 $v >> gpurun_out/r03s19/srv.log 2>&1 || exit $?
  BPSR_SERVER_COMBINE=0 timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 4 $v >> gpurun_out/r03s19/srv_nocomb.log 2>&1 || exit $?
done
timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 1 6 >> gpurun_out/r03s19/srv_1lane.log 2>&1 || exit $?
timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 8 6 >> gpurun_out/r03s19/srv_8lane.log 2>&1 || exit $?

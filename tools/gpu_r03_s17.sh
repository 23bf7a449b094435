export TMPDIR=/tmp; mkdir -p gpurun_out/r03s17
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/r03s17/prof -o run -- tools/server_cfg3_native tools/cfg3_resnet50_table.txt 6 4 4 > gpurun_out/r03s17/srv.log 2>&1; rc=$?
find gpurun_out/r03s17 -name '*.db' -delete
find gpurun_out/r03s17 -name '*_trace.csv' -size +1M -exec gzip -f {} \;
exit $rc

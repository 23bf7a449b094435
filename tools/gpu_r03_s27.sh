export TMPDIR=/tmp; mkdir -p gpurun_out/r03s27
OUT=gpurun_out/r03s27
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $OUT/prof -o run -- tools/server_cfg3_native tools/cfg3_resnet50_table.txt 6 4 8 > $OUT/srv8.log 2>&1; rc=$?
find $OUT -name '*.db' -delete
find $OUT -name '*_trace.csv' -size +1M -exec gzip -f {} \;
exit $rc

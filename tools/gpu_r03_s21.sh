export TMPDIR=/tmp; mkdir -p gpurun_out/r03s21
OUT=gpurun_out/r03s21
for v in 1 6 4 7 8; do
  timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 4 $v >> $OUT/srv.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_server_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/cfg3prof -o run -- tools/cfg3_native tools/cfg3_resnet50_table.txt 200 3 tools/cfg3_resnet50_tasks.txt inline_many > $OUT/cfg3prof.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/benchprof -o run -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $OUT/benchprof.log 2>&1; rc=$?
find $OUT -name '*.db' -delete
find $OUT -name '*_trace.csv' -size +1M -exec gzip -f {} \;
exit $rc

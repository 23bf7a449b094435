export TMPDIR=/tmp; mkdir -p gpurun_out/r03s50
OUT=gpurun_out/r03s50
timeout -k 10 900 python -u tools/bench_configs.py > $OUT/configs.log 2>&1; rc=$?
tail -3 $OUT/configs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 tools/cfg3_native tools/cfg3_resnet50_table.txt 200 7 tools/cfg3_resnet50_tasks.txt > $OUT/cfg3_native.jsonl 2>> $OUT/err.log || exit 1
timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 4 > $OUT/server_cfg3.jsonl 2>> $OUT/err.log || exit 1
timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 1 6 >> $OUT/server_cfg3.jsonl 2>> $OUT/err.log || exit 1
grep -c . $OUT/cfg3_native.jsonl $OUT/server_cfg3.jsonl

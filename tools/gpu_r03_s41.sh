export TMPDIR=/tmp; mkdir -p gpurun_out/r03s41
OUT=gpurun_out/r03s41
timeout -k 10 120 tools/cfg1_native 4 20 > $OUT/cfg1.jsonl 2> $OUT/err.log || { cat $OUT/err.log; exit 1; }
cat $OUT/cfg1.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace -o run -- tools/cfg1_native 4 6 1 > $OUT/trace.log 2>&1; rc=$?
find $OUT -name '*.db' -delete
ls -R $OUT/trace | head; exit $rc

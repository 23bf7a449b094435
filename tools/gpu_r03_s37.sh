export TMPDIR=/tmp; mkdir -p gpurun_out/r03s37
OUT=gpurun_out/r03s37
timeout -k 10 200 tools/hbm_probe3 256 20 > $OUT/p3_256.jsonl 2> $OUT/p3.err || { tail -5 $OUT/p3.err; exit 1; }
timeout -k 10 200 tools/hbm_probe3 528 10 > $OUT/p3_528.jsonl 2>> $OUT/p3.err || { tail -5 $OUT/p3.err; exit 1; }
cat $OUT/p3_256.jsonl $OUT/p3_528.jsonl

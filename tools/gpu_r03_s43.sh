export TMPDIR=/tmp; mkdir -p gpurun_out/r03s43
OUT=gpurun_out/r03s43
timeout -k 10 200 tools/hbm_probe2 528 > $OUT/p2_528.jsonl 2> $OUT/err.log || { cat $OUT/err.log; exit 1; }
timeout -k 10 200 tools/hbm_probe2 256 > $OUT/p2_256.jsonl 2>> $OUT/err.log || { cat $OUT/err.log; exit 1; }
cat $OUT/p2_528.jsonl $OUT/p2_256.jsonl

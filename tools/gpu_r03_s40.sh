export TMPDIR=/tmp; mkdir -p gpurun_out/r03s40
OUT=gpurun_out/r03s40
L=contig:0,sc-contig:0,contig:0,sc-contig:0,sc-contig:0,contig:0
PROBE3_LAYOUTS=$L timeout -k 10 200 tools/hbm_probe3 256 30 > $OUT/pre256.jsonl 2> $OUT/err.log || { cat $OUT/err.log; exit 1; }
PROBE3_LAYOUTS=$L timeout -k 10 200 tools/hbm_probe3 64 60 > $OUT/pre64.jsonl 2>> $OUT/err.log || { cat $OUT/err.log; exit 1; }
PROBE3_LAYOUTS=$L timeout -k 10 200 tools/hbm_probe3 16 100 > $OUT/pre16.jsonl 2>> $OUT/err.log || { cat $OUT/err.log; exit 1; }
cat $OUT/pre256.jsonl $OUT/pre64.jsonl $OUT/pre16.jsonl

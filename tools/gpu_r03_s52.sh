export TMPDIR=/tmp; mkdir -p gpurun_out/r03s52
OUT=gpurun_out/r03s52
timeout -k 10 300 python -u tools/zc_server_probe.py > $OUT/zc.jsonl 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
timeout -k 10 120 tools/cfg1_native 4 20 1 >> $OUT/zc.jsonl 2>> $OUT/err.log || exit 1
cut -c1-250 $OUT/zc.jsonl

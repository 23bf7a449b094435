export TMPDIR=/tmp; mkdir -p gpurun_out/r03s34
OUT=gpurun_out/r03s34
timeout -k 10 300 python -u tools/stride_probe.py --sizes 268435456 --aligns-kib 64 --pads-mib 0,256,768,1024,64,2,32 --rounds 2 > $OUT/spacing.jsonl 2> $OUT/spacing.err || { tail -5 $OUT/spacing.err; exit 1; }
cat $OUT/spacing.jsonl

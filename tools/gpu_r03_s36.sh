export TMPDIR=/tmp; mkdir -p gpurun_out/r03s36
OUT=gpurun_out/r03s36
timeout -k 10 600 python -u tools/interleave_probe.py > $OUT/interleave.jsonl 2> $OUT/interleave.err || { tail -5 $OUT/interleave.err; exit 1; }
cat $OUT/interleave.jsonl

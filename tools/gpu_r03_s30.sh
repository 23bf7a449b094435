export TMPDIR=/tmp; mkdir -p gpurun_out/r03s30
OUT=gpurun_out/r03s30
timeout -k 10 300 python -u tools/cumask_probe.py --keep 32,31,30,28,24,20,16 > $OUT/cumask.jsonl 2> $OUT/cumask.err; rc=$?
cat $OUT/cumask.jsonl; tail -3 $OUT/cumask.err; exit $rc

export TMPDIR=/tmp; mkdir -p gpurun_out/r03s39
OUT=gpurun_out/r03s39
timeout -k 10 500 python -u tools/skew_pattern_probe.py > $OUT/skewpat.jsonl 2> $OUT/skewpat.err || { tail -5 $OUT/skewpat.err; exit 1; }
tail -1 $OUT/skewpat.jsonl
for rep in 1 2 3; do for pf in 0 256; do
  BPSR_REC_PREFETCH=$pf timeout -k 10 200 tools/cfg3_native tools/cfg3_resnet50_table.txt 200 5 tools/cfg3_resnet50_tasks.txt host_release > $OUT/hr_pf$pf.$rep.jsonl 2>> $OUT/err.log || exit 1
done; done
grep -h -o '"variant": "[a-z_]*"\|"ms": [0-9.]*' $OUT/hr_pf*.jsonl | paste - - 

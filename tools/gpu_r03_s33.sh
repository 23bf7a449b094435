export TMPDIR=/tmp; mkdir -p gpurun_out/r03s33
OUT=gpurun_out/r03s33
for rep in 1 2; do for m in torch hipmalloc contiguous; do
  timeout -k 10 200 python -u tools/alloc_probe.py --method $m >> $OUT/alloc.jsonl 2>> $OUT/alloc.err || { tail -5 $OUT/alloc.err; exit 1; }
done; done
cat $OUT/alloc.jsonl

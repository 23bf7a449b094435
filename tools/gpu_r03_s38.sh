export TMPDIR=/tmp; mkdir -p gpurun_out/r03s38
OUT=gpurun_out/r03s38
# correctness first: the suites that run batched launches, plans and block queues
timeout -k 10 600 python -u -m pytest tests/test_blockq_gpu.py tests/test_parity_gpu.py tests/test_pushloop_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
# A/B: record prefetch off / on, twice, same box
for rep in 1 2; do for pf in 0 256; do
  BPSR_REC_PREFETCH=$pf timeout -k 10 200 tools/cfg3_native tools/cfg3_resnet50_table.txt 200 5 tools/cfg3_resnet50_tasks.txt plan_all,pre_released,inline_many,host_release > $OUT/cfg3_pf$pf.$rep.jsonl 2>> $OUT/err.log || exit 1
  BPSR_REC_PREFETCH=$pf timeout -k 10 200 python -u tools/interleave_probe.py --sizes 268435456 --chunks-kib 16384,1024 --rounds 1 > $OUT/plan256_pf$pf.$rep.jsonl 2>> $OUT/err.log || exit 1
done; done
for f in $OUT/cfg3_pf*.jsonl $OUT/plan256_pf*.jsonl; do echo "== $f"; cut -c1-220 $f; done

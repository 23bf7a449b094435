export TMPDIR=/tmp; mkdir -p gpurun_out/r03s53
OUT=gpurun_out/r03s53
timeout -k 10 600 python -u -m pytest tests/test_server_gpu.py tests/test_parity_gpu.py -k "batched or plan or prefetch or many or view" -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for pf in 0 256; do
  BPSR_REC_PREFETCH=$pf timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 4 4 > $OUT/srv4_pf$pf.$rep.jsonl 2>> $OUT/err.log || exit 1
  BPSR_REC_PREFETCH=$pf timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 1 6 > $OUT/srv6_pf$pf.$rep.jsonl 2>> $OUT/err.log || exit 1
done; done
for f in $OUT/srv*.jsonl; do echo "$f $(grep -o '"round_ms": [0-9.]*' $f)"; done

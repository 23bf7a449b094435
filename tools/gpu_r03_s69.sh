export TMPDIR=/tmp; mkdir -p gpurun_out/r03s69
OUT=gpurun_out/r03s69
BPSR_SERVER_SPIN_US=50 timeout -k 10 900 python -u -m pytest tests/test_server_gpu.py tests/test_server_group_gpu.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for sp in 0 20 100; do
    for v in 0 1; do
      BPSR_SERVER_SPIN_US=$sp timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 10 4 $v > $OUT/srv_v$v.sp$sp.$rep.jsonl 2>> $OUT/err.log || exit 1
    done
  done
done
for f in $OUT/srv*.jsonl; do python -c "
import json
for l in open('$f'):
    r=json.loads(l); print('$f'.split('/')[-1].ljust(22), r['variant'].ljust(12), r['round_ms'], r['min_ms'], r['pulls_agree'])"; done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/full.log 2>&1; rc=$?; tail -2 $OUT/full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log

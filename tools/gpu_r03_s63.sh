export TMPDIR=/tmp; mkdir -p gpurun_out/r03s63
OUT=gpurun_out/r03s63
timeout -k 10 900 python -u -m pytest tests/test_server_gpu.py tests/test_server_group_gpu.py tests/test_native_gpu.py tests/test_knownanswer_gpu.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
ALT=$PWD/prophet_amd/alt
for rep in 1 2; do for lib in new old; do
  if [ $lib = old ]; then export LD_LIBRARY_PATH=$ALT; else unset LD_LIBRARY_PATH; fi
  for v in 0 1; do
    timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 10 4 $v > $OUT/srv_v${v}_$lib.$rep.jsonl 2>> $OUT/err.log || exit 1
  done
  timeout -k 10 120 tools/cfg1_native 4 10 0 > $OUT/cfg1_$lib.$rep.jsonl 2>> $OUT/err.log || exit 1
done; done
unset LD_LIBRARY_PATH
for f in $OUT/srv*.jsonl $OUT/cfg1*.jsonl; do python -c "
import json
for l in open('$f'):
    r=json.loads(l); print('$f'.split('/')[-1].ljust(22), r.get('variant', r.get('pulls',''))[:40].ljust(42), r['round_ms'], r.get('pulls_agree', r.get('exact')))"; done

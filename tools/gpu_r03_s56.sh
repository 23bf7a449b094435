export TMPDIR=/tmp; mkdir -p gpurun_out/r03s56
OUT=gpurun_out/r03s56
timeout -k 10 900 python -u -m pytest tests/test_blockq_gpu.py tests/test_parity_gpu.py tests/test_pushloop_gpu.py tests/test_server_gpu.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
ALT=$PWD/prophet_amd/alt
for rep in 1 2; do for lib in new old; do
  if [ $lib = old ]; then export LD_LIBRARY_PATH=$ALT; else unset LD_LIBRARY_PATH; fi
  timeout -k 10 200 tools/cfg3_native tools/cfg3_resnet50_table.txt 200 5 tools/cfg3_resnet50_tasks.txt plan_all,pre_released,inline_many > $OUT/cfg3_$lib.$rep.jsonl 2>> $OUT/err.log || exit 1
  CFG3_PRIORITY_CONSUMER=1 timeout -k 10 200 tools/cfg3_native tools/cfg3_resnet50_table.txt 200 5 tools/cfg3_resnet50_tasks.txt pre_released > $OUT/cfg3cs_$lib.$rep.jsonl 2>> $OUT/err.log || exit 1
  timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 1 6 > $OUT/srv_$lib.$rep.jsonl 2>> $OUT/err.log || exit 1
done; done
unset LD_LIBRARY_PATH
for f in $OUT/cfg3*.jsonl $OUT/srv*.jsonl; do python -c "
import json
for l in open('$f'):
    r=json.loads(l); print('$f'.split('/')[-1].ljust(22), r['variant'][:40].ljust(42), r.get('ms', r.get('round_ms')), r.get('exact_vs_plan', r.get('pulls_agree')))"; done

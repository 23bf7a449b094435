export TMPDIR=/tmp; mkdir -p gpurun_out/r03s57
OUT=gpurun_out/r03s57
ALT=$PWD/prophet_amd/alt
for rep in 1 2 3 4; do for lib in new old; do
  if [ $lib = old ]; then export LD_LIBRARY_PATH=$ALT; else unset LD_LIBRARY_PATH; fi
  timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 1 6 > $OUT/srv1_$lib.$rep.jsonl 2>> $OUT/err.log || exit 1
  timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 4 4 > $OUT/srv4_$lib.$rep.jsonl 2>> $OUT/err.log || exit 1
done; done
unset LD_LIBRARY_PATH
for f in $OUT/srv*.jsonl; do python -c "
import json
for l in open('$f'):
    r=json.loads(l); print('$f'.split('/')[-1].ljust(22), r['variant'][:40].ljust(42), r['round_ms'], r['min_ms'], r['fold_launches_per_round'], r['pulls_agree'])"; done

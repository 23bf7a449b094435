export TMPDIR=/tmp; mkdir -p gpurun_out/r03s59
OUT=gpurun_out/r03s59
for rep in 1 2 3; do for inf in 1 2 4; do
  BPSR_SERVER_INFLIGHT=$inf timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 1 6 > $OUT/s1_i$inf.$rep.jsonl 2>> $OUT/err.log || exit 1
  BPSR_SERVER_INFLIGHT=$inf timeout -k 10 200 tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 4 4 > $OUT/s4_i$inf.$rep.jsonl 2>> $OUT/err.log || exit 1
done; done
for f in $OUT/s*.jsonl; do python -c "
import json
for l in open('$f'):
    r=json.loads(l); print('$f'.split('/')[-1].ljust(16), r['variant'][:30].ljust(32), r['round_ms'], r['min_ms'], r['fold_launches_per_round'], r['pulls_agree'])"; done

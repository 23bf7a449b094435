export TMPDIR=/tmp; mkdir -p gpurun_out/r03s46
OUT=gpurun_out/r03s46
timeout -k 10 200 tools/event_probe 1,4,16,64,256 100 > $OUT/evprobe.jsonl 2> $OUT/err.log || { cat $OUT/err.log; exit 1; }
python -c "
import json
for l in open('$OUT/evprobe.jsonl'):
    r=json.loads(l); print(r['mib_per_source'], r['marker'].ljust(10), r['round'], r['us_per_fold_avg'], r['us_per_fold_best'])"

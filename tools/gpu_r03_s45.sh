export TMPDIR=/tmp; mkdir -p gpurun_out/r03s45
OUT=gpurun_out/r03s45
timeout -k 10 300 python -u tools/event_scope_probe.py > $OUT/evscope.jsonl 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
python -c "
import json
for l in open('$OUT/evscope.jsonl'):
    r=json.loads(l); print(r['bytes_per_source'], r['event'], r['round'], r['us_per_fold'])"

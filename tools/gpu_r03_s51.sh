export TMPDIR=/tmp; mkdir -p gpurun_out/r03s51
OUT=gpurun_out/r03s51
for mib in 256 320 384 448 512 528 640; do
  PROBE_XMAP=1 timeout -k 10 200 tools/hbm_probe2 $mib > $OUT/x$mib.jsonl 2>> $OUT/err.log || { cat $OUT/err.log; exit 1; }
done
python - <<'PY'
import json,collections
for mib in (256,320,384,448,512,528,640):
    d=collections.defaultdict(list)
    for l in open(f'gpurun_out/r03s51/x{mib}.jsonl'):
        r=json.loads(l); d[r['v'].replace('n8_v2_wg1cu','id').replace('id_xcd','')].append(r['ms'])
    print(mib, {k: [round(x,4) for x in v] for k,v in d.items()})
PY

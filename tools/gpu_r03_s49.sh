export TMPDIR=/tmp; mkdir -p gpurun_out/r03s49
OUT=gpurun_out/r03s49
L=contig:0,multi:2,multi:4,pipe:2,pipe:4,contig:0,multi:2,multi:4,pipe:2,pipe:4
PROBE3_LAYOUTS=$L timeout -k 10 200 tools/hbm_probe3 256 30 > $OUT/m256.jsonl 2> $OUT/err.log || { cat $OUT/err.log; exit 1; }
PROBE3_LAYOUTS=$L timeout -k 10 200 tools/hbm_probe3 64 60 > $OUT/m64.jsonl 2>> $OUT/err.log || { cat $OUT/err.log; exit 1; }
python -c "
import json
for f in ('m256','m64'):
    for l in open('$OUT/'+f+'.jsonl'):
        r=json.loads(l); print(f, r['tiles_per_wg'], r['pipelined'], r['ms_avg'], r['frac_avg'])"

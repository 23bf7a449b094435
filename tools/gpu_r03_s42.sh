export TMPDIR=/tmp; mkdir -p gpurun_out/r03s42
OUT=gpurun_out/r03s42
for l in 1 2 4 8; do for m in 0 1; do
  timeout -k 10 120 tools/cfg1_native $l 20 $m >> $OUT/lanes.jsonl 2>> $OUT/err.log || { cat $OUT/err.log; exit 1; }
done; done
BPSR_SERVER_PULL_COPY=kernel timeout -k 10 120 tools/cfg1_native 4 20 0 >> $OUT/lanes.jsonl 2>> $OUT/err.log || exit 1
BPSR_SERVER_COMBINE=0 timeout -k 10 120 tools/cfg1_native 4 20 0 >> $OUT/lanes.jsonl 2>> $OUT/err.log || exit 1
BPSR_SERVER_COMBINE=0 timeout -k 10 120 tools/cfg1_native 4 20 1 >> $OUT/lanes.jsonl 2>> $OUT/err.log || exit 1
python -c "
import json
for l in open('$OUT/lanes.jsonl'):
    r=json.loads(l); print(r['lanes'], r['pulls'][15:], r['round_ms'], r['min_ms'], r['gibps'], r['exact'])"
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace0 -o run -- tools/cfg1_native 4 6 0 > $OUT/trace.log 2>&1; rc=$?
find $OUT -name '*.db' -delete
exit $rc

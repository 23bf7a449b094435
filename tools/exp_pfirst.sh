set -u
O=gpurun_out/r02s98
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_blockq_gpu.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for r in 1 2 3; do for p in 0 1; do
  t=p${p}_r$r
  BPSR_PARTIAL_FIRST=$p timeout -k 10 120 ./tools/cfg3_native tools/cfg3_resnet50_table.txt 200 5 "" > $O/c_$t.jsonl 2>$O/c_$t.err || { echo "cfg3 $t rc=$?"; tail $O/c_$t.err; exit 1; }
  python -c "
import json
c=[json.loads(l) for l in open('$O/c_$t.jsonl') if l.startswith('{')]
print('$t', [(x['variant'].replace('blockq_','')[:14], x['ms'], x['exact_vs_plan']) for x in c])"
done; done

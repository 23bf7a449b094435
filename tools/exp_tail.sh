set -u
O=gpurun_out/r02s89
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for cfg in "0 1" "512 2" "512 4" "1024 2" "256 4" "1024 4"; do
  set -- $cfg
  t=k$1_d$2_r$r
  BPSR_TAIL_TILES=$1 BPSR_TAIL_DIV=$2 timeout -k 10 120 ./tools/cfg3_native tools/cfg3_resnet50_table.txt 200 5 "" blockq_ > $O/cfg3_$t.jsonl 2>$O/cfg3_$t.err || { echo "cfg3 $t rc=$?"; tail $O/cfg3_$t.err; exit 1; }
  BPSR_TAIL_TILES=$1 BPSR_TAIL_DIV=$2 timeout -k 10 120 ./tools/cfg3_native tools/cfg3_resnet50_table.txt 200 5 "" plan_ > $O/plan_$t.jsonl 2>$O/plan_$t.err || { echo "plan $t rc=$?"; tail $O/plan_$t.err; exit 1; }
  python - "$O" "$t" <<'PY'
import json,sys
O,t=sys.argv[1:3]
c=[json.loads(l) for l in open(f'{O}/cfg3_{t}.jsonl') if l.startswith('{')]+[json.loads(l) for l in open(f'{O}/plan_{t}.jsonl') if l.startswith('{')]
print(t, [(x['variant'].replace('blockq_',''), x['ms'], x['exact_vs_plan']) for x in c])
PY
done; done
BPSR_TAIL_TILES=512 BPSR_TAIL_DIV=4 timeout -k 10 200 python bench.py --steps 5 --no-cpu-baseline --no-scaling --no-fp16 --no-e2e > $O/bench_split.json 2> $O/bench_split.err || { echo "bench rc=$?"; tail $O/bench_split.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_split.json')); print(d['cfg3_blockq'])"

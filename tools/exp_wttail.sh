set -u
O=gpurun_out/r02s90
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do for k in 0 2048 4096 8192; do
  t=k${k}_r$r
  BPSR_WT_TAIL_TILES=$k timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-cfg3 --no-fp16 --no-e2e > $O/bench_$t.json 2>$O/bench_$t.err || { echo "bench $t rc=$?"; tail $O/bench_$t.err; exit 1; }
  BPSR_WT_TAIL_TILES=$k timeout -k 10 200 python tools/occ_sweep.py --mib 128,192 --occ 1 --vpt 2 > $O/occ_$t.jsonl 2>$O/occ_$t.err || { echo "occ $t rc=$?"; exit 1; }
  python -c "
import json
b=json.load(open('$O/bench_$t.json')); o=[json.loads(l) for l in open('$O/occ_$t.jsonl')]
print('$t', b['roofline']['kernel_ms'], b['roofline']['frac'], b['check_vs_torch_fold'], b['scaling_cfg4']['g1_fold_ms'], [x['us'] for x in o])"
done; done

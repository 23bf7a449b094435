set -u
O=gpurun_out/r02s87
mkdir -p $O
export TMPDIR=/tmp
run() { # tag wtmib
  local t=$1
  export BPSR_WT_MAX_MIB=$2
  timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-cfg3 --no-fp16 --no-e2e > $O/bench_$t.json 2>$O/bench_$t.err || { echo "bench $t rc=$?"; tail $O/bench_$t.err; exit 1; }
  timeout -k 10 200 python tools/occ_sweep.py --mib 16,33,48,66,80 --occ 1 --vpt 2 > $O/occ_$t.jsonl 2>$O/occ_$t.err || { echo "occ $t rc=$?"; tail $O/occ_$t.err; exit 1; }
  timeout -k 10 120 ./tools/cfg3_native tools/cfg3_resnet50_table.txt 200 5 "" blockq_ > $O/cfg3_$t.jsonl 2>$O/cfg3_$t.err || { echo "cfg3 $t rc=$?"; tail $O/cfg3_$t.err; exit 1; }
}
for r in 1 2 3; do run N$r 0 && run W$r 96; done
python - <<'PY'
import json
O='gpurun_out/r02s87'
for t in ('N1','W1','N2','W2','N3','W3'):
    b=json.loads(open(f'{O}/bench_{t}.json').read())
    occ=[json.loads(l) for l in open(f'{O}/occ_{t}.jsonl')]
    c3=[json.loads(l) for l in open(f'{O}/cfg3_{t}.jsonl') if l.startswith('{')]
    print(t, 'head', b['roofline']['kernel_ms'], b['check_vs_torch_fold'], 'g1', b['scaling_cfg4']['g1_fold_ms'],
          'occ', [o['us'] for o in occ], 'cfg3', [(c['ms'], c['exact_vs_plan']) for c in c3])
PY

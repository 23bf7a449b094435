set -u
O=gpurun_out/r02s85
mkdir -p $O
export TMPDIR=/tmp
run() { # tag dir
  local t=$1 d=$2
  (cd $d && timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-cfg3 --no-fp16 --no-e2e) > $O/bench_$t.json 2>$O/bench_$t.err || { echo "bench $t rc=$?"; tail $O/bench_$t.err; exit 1; }
  (cd $d && timeout -k 10 200 python tools/occ_sweep.py --mib 16,33,66,128 --occ 1 --vpt 2) > $O/occ_$t.jsonl 2>$O/occ_$t.err || { echo "occ $t rc=$?"; tail $O/occ_$t.err; exit 1; }
  (cd $d && timeout -k 10 120 ./tools/cfg3_native tools/cfg3_resnet50_table.txt 200 5 "" blockq_) > $O/cfg3_$t.jsonl 2>$O/cfg3_$t.err || { echo "cfg3 $t rc=$?"; tail $O/cfg3_$t.err; exit 1; }
}
for r in 1 2; do run A$r . && run B$r r02ab; done
python - <<'PY'
import json
O='gpurun_out/r02s85'
for t in ('A1','B1','A2','B2'):
    b=json.loads(open(f'{O}/bench_{t}.json').read())
    occ=[json.loads(l) for l in open(f'{O}/occ_{t}.jsonl')]
    c3=[json.loads(l) for l in open(f'{O}/cfg3_{t}.jsonl') if l.startswith('{')]
    print(t, 'head', b['roofline']['kernel_ms'], b['roofline']['frac'], b['check_vs_torch_fold'], 'cfg4g1', b['scaling_cfg4']['g1_fold_ms'],
          'occ', [(o['mib'], o['us']) for o in occ], 'cfg3', [(c['variant'][7:], c['ms'], c['exact_vs_plan']) for c in c3])
PY

set -u
O=gpurun_out/r02s86
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do for t in A B; do
  d=.; [ $t = B ] && d=r02ab
  (cd $d && timeout -k 10 300 python tools/occ_sweep.py --mib 4,8,24,48,80,96,112,160,192,256,384,527.8 --occ 1 --vpt 2) > $O/occ_$t$r.jsonl 2>$O/occ_$t$r.err || { echo "occ $t rc=$?"; tail $O/occ_$t$r.err; exit 1; }
done; done
python - <<'PY'
import json
O='gpurun_out/r02s86'
res={}
for t in ('A1','B1','A2','B2'):
    for l in open(f'{O}/occ_{t}.jsonl'):
        d=json.loads(l); res.setdefault(d['mib'],{})[t]=d['us']
for m,v in sorted(res.items()):
    a=(v['A1']+v['A2'])/2; b=(v['B1']+v['B2'])/2
    print(m, v, 'B/A=%.4f'%(b/a))
PY

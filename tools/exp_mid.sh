set -u
mkdir -p gpurun_out/r02s83
export TMPDIR=/tmp
for r in 1 2; do
timeout -k 10 300 python tools/occ_sweep.py --mib 48,56,64,65.974,72,80,88,96,128 --occ 1 --vpt 2,4 > gpurun_out/r02s83/mid_$r.jsonl 2> gpurun_out/r02s83/mid_$r.err || { echo "rc=$?"; tail gpurun_out/r02s83/mid_$r.err; exit 1; }
done
python - <<'PY'
import json
for r in (1,2):
    for l in open(f'gpurun_out/r02s83/mid_{r}.jsonl'):
        d=json.loads(l); print(r, d['mib'], d['occ'], d['vpt'], d['us'], d['GBps'])
PY

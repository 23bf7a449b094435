export TMPDIR=/tmp; mkdir -p gpurun_out/r03s35
OUT=gpurun_out/r03s35
P=$(python -c "print(','.join(str(x) for x in [0,1,4,8,16]+list(range(32,1057,32))))")
timeout -k 10 500 python -u tools/stride_probe.py --sizes 268435456 --aligns-kib 64 --pads-mib $P --rounds 1 --reps 15 > $OUT/spacing256.jsonl 2> $OUT/spacing.err || { tail -5 $OUT/spacing.err; exit 1; }
P2=$(python -c "print(','.join(str(x) for x in range(0,545,32)))")
timeout -k 10 400 python -u tools/stride_probe.py --sizes 553430176 --aligns-kib 64 --pads-mib $P2 --rounds 1 --reps 10 > $OUT/spacing553.jsonl 2>> $OUT/spacing.err || { tail -5 $OUT/spacing.err; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/r03s35/spacing256.jsonl","gpurun_out/r03s35/spacing553.jsonl"):
    for l in open(f):
        r=json.loads(l); print(r["bucket_bytes"], r["pad_mib"], r["stride"], r["frac"])
PY

export TMPDIR=/tmp; mkdir -p gpurun_out/r03s31
OUT=gpurun_out/r03s31
timeout -k 10 400 python -u tools/stride_probe.py > $OUT/stride.jsonl 2> $OUT/stride.err || { tail -5 $OUT/stride.err; exit 1; }
timeout -k 10 200 python -u bench.py --steps 50 --no-cpu-baseline --no-cfg3 --no-e2e --no-fp16 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/stride.jsonl; python -c "import json;l=json.load(open('$OUT/bench.json'));print(l['roofline'])"

export TMPDIR=/tmp; mkdir -p gpurun_out/r03s32
OUT=gpurun_out/r03s32
timeout -k 10 500 python -u tools/chunk_probe.py > $OUT/chunk.jsonl 2> $OUT/chunk.err || { tail -5 $OUT/chunk.err; exit 1; }
timeout -k 10 200 python -u bench.py --steps 50 --no-cpu-baseline --no-cfg3 --no-e2e --no-fp16 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/chunk.jsonl; python -c "import json;l=json.load(open('$OUT/bench.json'));r=l['roofline'];print(r['frac'],r['kernel_ms'],r['kernel_ms_blocks'],l['ms_per_step'])"

export TMPDIR=/tmp; mkdir -p gpurun_out/r03s62
OUT=gpurun_out/r03s62
timeout -k 10 600 python -u -m pytest tests/test_bench_gpu.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --gpus 8 --rehearse-one-gpu --steps 20 --warmup 3 > $OUT/bench_w8.json 2> $OUT/bench_w8.err; rc=$?
python -c "
import json;l=json.load(open('$OUT/bench_w8.json'))
print(l['n_gpus'], l.get('error'), l['device']); print(json.dumps(l['scaling_cfg4'].get('scatter'))[:400]); print(json.dumps(l.get('local_reduce'))[:500])"
exit $rc

export TMPDIR=/tmp; mkdir -p gpurun_out/r03s60
OUT=gpurun_out/r03s60
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/benchprof -o run -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-scaling --no-fp16 --no-cfg3 --no-e2e > $OUT/benchprof.json 2> $OUT/benchprof.err; rc=$?
find $OUT -name '*.db' -delete
find $OUT -name '*_trace.csv' -size +1M -exec gzip -f {} \;
python -c "import json;l=json.load(open('$OUT/bench.json'));r=l['roofline'];print(l['value'],r['frac'],l['cfg3_blockq']['live']['frac_of_roofline'],l['fp16']['frac_of_roofline'])"
grep fold_kernel $OUT/benchprof/run_kernel_stats.csv | head -3; python -c "import json;print(json.load(open('$OUT/benchprof.json'))['roofline']['kernel_ms'])"
exit $rc

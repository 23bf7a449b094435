export TMPDIR=/tmp; mkdir -p gpurun_out/r03s68
OUT=gpurun_out/r03s68
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
python -c "import json;l=json.load(open('$OUT/bench.json'));r=l['roofline'];print(l['value'],r['frac'],l['cfg3_blockq']['live']['frac_of_roofline'],l['fp16']['frac_of_roofline'])"

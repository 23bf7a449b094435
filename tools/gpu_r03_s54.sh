export TMPDIR=/tmp; mkdir -p gpurun_out/r03s54
OUT=gpurun_out/r03s54
for rep in 1 2; do
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests$rep.log 2>&1; rc=$?; tail -2 $OUT/tests$rep.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
python -c "import json;l=json.load(open('$OUT/bench.json'));r=l['roofline'];print(l['value'],r['frac'],l['cfg3_blockq']['live']['frac_of_roofline'],l['fp16']['frac_of_roofline'],l['scaling_cfg4']['per_gpu_frac_of_roofline'],l['e2e_cfg5']['node_e2e_GiBps'],l['cpu_baseline']['value'])"

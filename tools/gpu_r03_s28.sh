export TMPDIR=/tmp; mkdir -p gpurun_out/r03s28
OUT=gpurun_out/r03s28
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || exit $?
tail -1 $OUT/bench.log

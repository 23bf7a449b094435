export TMPDIR=/tmp; mkdir -p gpurun_out/r03s24
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r03s24/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03s24/tests.log; exit $rc

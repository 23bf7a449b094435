export TMPDIR=/tmp; mkdir -p gpurun_out/r03s13
timeout -k 10 400 python -u -m pytest tests/test_pushloop_gpu.py tests/test_blockq_gpu.py -m gpu -x -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r03s13/tests.log 2>&1; rc=$?; tail -5 gpurun_out/r03s13/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/cfg3_native tools/cfg3_resnet50_table.txt 200 7 tools/cfg3_resnet50_tasks.txt > gpurun_out/r03s13/cfg3.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03s13/bench.log 2>&1; rc=$?; tail -c 3000 gpurun_out/r03s13/bench.log; exit $rc

export TMPDIR=/tmp; mkdir -p gpurun_out/r03s11
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py tests/test_shard_abi_gpu.py tests/test_shard_gpu.py tests/test_torch_ops.py -m gpu -x -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r03s11/tests.log 2>&1; rc=$?; tail -5 gpurun_out/r03s11/tests.log
[ $rc -le 1 ] || exit $rc
bash tools/gpu_r03.sh r03s11 srvall srvprof cfg3prof

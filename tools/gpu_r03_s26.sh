export TMPDIR=/tmp; mkdir -p gpurun_out/r03s26
OUT=gpurun_out/r03s26
timeout -k 10 500 python tools/pmc_traffic.py --out $OUT/pmc --session r03s26 > $OUT/pmc.log 2>&1 || exit $?
find $OUT -name '*.db' -delete
timeout -k 10 900 python tools/bench_configs.py > $OUT/configs.log 2>&1; rc=$?
exit $rc

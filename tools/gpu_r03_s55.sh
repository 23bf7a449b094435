export TMPDIR=/tmp; mkdir -p gpurun_out/r03s55
OUT=gpurun_out/r03s55
timeout -s KILL 300 python -u tools/pmc_cfg3.py $OUT/pmc_cfg3 > $OUT/pmc_cfg3.log 2>&1; rc=$?
find $OUT -name '*.db' -delete
find $OUT -name '*_trace.csv' -size +1M -exec gzip -f {} \;
tail -3 $OUT/pmc_cfg3.log; exit $rc

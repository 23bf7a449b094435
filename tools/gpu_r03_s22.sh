export TMPDIR=/tmp; mkdir -p gpurun_out/r03s22
OUT=gpurun_out/r03s22
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/benchprof -o run -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-scaling --no-fp16 --no-cfg3 --no-e2e > $OUT/benchprof.log 2>&1; rc=$?
echo "benchprof rc=$rc" >> $OUT/steps.log
find $OUT -name '*.db' -delete
find $OUT -name '*_trace.csv' -size +1M -exec gzip -f {} \;
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/cfg3benchprof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-scaling --no-fp16 --no-e2e > $OUT/cfg3benchprof.log 2>&1; rc=$?
echo "cfg3benchprof rc=$rc" >> $OUT/steps.log
find $OUT -name '*.db' -delete
find $OUT -name '*_trace.csv' -size +1M -exec gzip -f {} \;
exit $rc

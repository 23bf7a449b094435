export TMPDIR=/tmp; mkdir -p gpurun_out/r03s29
OUT=gpurun_out/r03s29
# world-8 rehearsal: 8 rank processes through bench.py's own launcher, all on cuda:0 (gloo)
timeout -k 10 500 python -u bench.py --gpus 8 --rehearse-one-gpu --steps 20 --warmup 3 > $OUT/bench_w8.json 2> $OUT/bench_w8.err; rc=$?
tail -c 3000 $OUT/bench_w8.json; tail -5 $OUT/bench_w8.err; exit $rc

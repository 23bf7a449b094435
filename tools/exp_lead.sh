set -u
O=gpurun_out/r02s93
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail $O/bench.err; exit 1; }
python -c "
import json; b=json.load(open('$O/bench.json')); print(b['roofline']['kernel_ms'], b['roofline']['frac'], b['ms_per_step']); print(b['scaling_cfg4']); print(b['cfg3_blockq']['live'], b['cfg3_blockq']['pre_released'])"
timeout -k 10 300 python tools/bench_configs.py --only cfg4 > $O/cfg4.jsonl 2> $O/cfg4.err || { echo "cfg4 rc=$?"; tail $O/cfg4.err; exit 1; }
cat $O/cfg4.jsonl | cut -c1-160
timeout -k 10 300 python -u -m pytest tests/test_bench_gpu.py -x -q --timeout 280 --timeout-method thread > $O/tbench.log 2>&1 || { echo "tbench rc=$?"; tail $O/tbench.log; exit 1; }
tail -1 $O/tbench.log

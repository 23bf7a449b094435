set -u
O=gpurun_out/r02s95
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_torch_ops.py tests/test_pipeline_gpu.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 300 python tools/graph_vs_eager.py 69178772,69206016,138357544,276715088,268435456,4096000,16777220 > $O/eager.jsonl 2>$O/eager.err || { echo "eager rc=$?"; tail $O/eager.err; exit 1; }
cut -c1-60 $O/eager.jsonl

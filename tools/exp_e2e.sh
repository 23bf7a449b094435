set -u
mkdir -p gpurun_out/r02s82
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-cfg3 --no-fp16 --no-scaling > gpurun_out/r02s82/n1.json 2> gpurun_out/r02s82/n1.err || { echo "rc=$?"; tail -20 gpurun_out/r02s82/n1.err; exit 1; }
cat gpurun_out/r02s82/n1.json
timeout -k 10 300 python bench.py --gpus 2 --rehearse-one-gpu --steps 20 --no-cpu-baseline --no-scaling > gpurun_out/r02s82/n2r.json 2> gpurun_out/r02s82/n2r.err || { echo "rc=$?"; tail -20 gpurun_out/r02s82/n2r.err; exit 1; }
cat gpurun_out/r02s82/n2r.json

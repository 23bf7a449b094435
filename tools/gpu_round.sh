#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, tuning sweep, rocprof kernel
# trace.  Each GPU step has its own time limit; the script stops at the first
# step that ends in anything other than success or an ordinary test failure
# (fault, abort, segfault, timeout).  Output: gpurun_out/<tag>/...
#   usage: tools/gpu_round.sh <tag> [steps...]   steps: test smoke bench sweep prof pmc occ cfg3 configs cfg1 lat cfg3trace
set -u
TAG=${1:-r01}; shift || true
STEPS=${*:-"test smoke bench sweep prof"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0

run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))" | tee -a "$OUT/steps.log"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)" | tee -a "$OUT/steps.log"
    exit $rc
  fi
  return 0
}

for s in $STEPS; do
  case $s in
    test)  run pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 ;;
    blockq) run blockq 300 python -u -m pytest tests/test_blockq_gpu.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    torchops) run torchops 300 python -u -m pytest tests/test_torch_ops.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    cfg3only) run cfg3only 300 python tools/bench_configs.py --only cfg3 ;;
    batchocc) for o in 0 2 4; do
             run batch_occ$o 300 env BPSR_SMALL_OCC_BATCH=$o python tools/bench_configs.py --only cfg3 || exit 1
           done ;;
    gateocc) for o in 1 2 3; do
             run gate_occ$o 300 env BPSR_BQ_GATE_OCC=$o python tools/bench_configs.py --only cfg3 --variants blockq || exit 1
           done ;;
    bqexp) for v in 1 2 4; do
             run bqexp_v$v 300 env BPSR_BQ_VPT=$v python tools/bench_configs.py --only cfg3 --variants blockq || exit 1
           done ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    sweep) run sweep 600 python tools/sweep.py ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$OUT/prof" -o bench -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline ;;
    pmc)   run pmc 900 python tools/pmc_traffic.py --out "$OUT/pmc" ;;
    occ)   run occ 600 python tools/occ_sweep.py ;;
    cfg3)  run cfg3 600 python tools/bench_configs.py --only cfg3,sweep ;;
    configs) run configs 900 python tools/bench_configs.py ;;
    dtypes) run bench_f16 300 python bench.py --dtype f16 --no-cpu-baseline &&
            run bench_bf16 300 python bench.py --dtype bf16 --no-cpu-baseline &&
            run bench_bf16_16 300 python bench.py --dtype bf16 --workers 16 --no-cpu-baseline &&
            run bench_f32_16 300 python bench.py --workers 16 --no-cpu-baseline &&
            run bench_f32_2 300 python bench.py --workers 2 --no-cpu-baseline ;;
    nsweep) for n in 2 3 4 16; do
              run nsweep_$n 400 python tools/occ_sweep.py --workers $n --mib 64,256 --occ 1,2,4,8 --vpt 1,2,4 || exit 1
            done ;;
    ops)   run ops 300 python tools/op_probe.py &&
           for d in f64 i32 i64 u8 i8; do run bench_$d 300 python bench.py --dtype $d --no-cpu-baseline || exit 1; done &&
           run bench_f16acc 300 python bench.py --dtype f16 --mode accum --no-cpu-baseline &&
           run bench_bf16acc 300 python bench.py --dtype bf16 --mode accum --no-cpu-baseline ;;
    copysweep) for o in 0 2 4 8; do for v in 2 4; do
                 run copy_o${o}_v$v 120 env BPSR_COPY_OCC=$o BPSR_COPY_VPT=$v python tools/op_probe.py --mib 256 || exit 1
                 run copy64_o${o}_v$v 120 env BPSR_COPY_OCC=$o BPSR_COPY_VPT=$v python tools/op_probe.py --mib 64 || exit 1
               done; done ;;
    acc)   run bench_f16acc 300 python bench.py --dtype f16 --mode accum --no-cpu-baseline &&
           run bench_bf16acc 300 python bench.py --dtype bf16 --mode accum --no-cpu-baseline &&
           run ops 300 python tools/op_probe.py ;;
    cfg1)  run cfg1 300 python tools/bench_configs.py --only cfg1 ;;
    server) run server 300 python -u -m pytest tests/test_server_gpu.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    lat)   run lat 300 python tools/latency_probe.py ;;
    cfg3p) run cfg3p 300 python tools/cfg3_probe.py ;;
    thr)   for t in 2048 4096 8192 1000000; do
             run thr_b$t 300 env BPSR_OCC_MIN_TILES_BATCH=$t python tools/cfg3_probe.py --occ 1 --streams 1
           done
           for t in 2048 4096 8192; do
             run thr_f$t 300 env BPSR_OCC_MIN_TILES=$t python tools/occ_sweep.py --mib 8,16,32,64,128 --occ 1 --vpt 2,4
           done ;;
    cfg3trace) run cfg3trace 600 rocprofv3 --kernel-trace --output-format csv \
             -d "$OUT/cfg3trace" -o cfg3 -- python tools/bench_configs.py --only cfg3 ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "done"

#!/bin/bash
# Round-2 GPU session steps.  Each GPU step has its own time limit; the script
# stops at the first step that ends in anything other than success or an
# ordinary test failure (fault, abort, segfault, timeout).
#   usage: tools/gpu_r02.sh <tag> <steps...>
set -u
TAG=${1:-r02}; shift || true
STEPS=${*:-"gputest"}
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
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)" | tee -a "$OUT/steps.log"
    exit $rc
  fi
  return 0
}

for s in $STEPS; do
  case $s in
    gputest) run gputest 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    blockq) run blockq 400 python -u -m pytest tests/test_blockq_gpu.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    server) run server 400 python -u -m pytest tests/test_server_gpu.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    cfg3n) run cfg3_native 300 ./tools/cfg3_native tools/cfg3_resnet50_table.txt 200 7 tools/cfg3_resnet50_tasks.txt ;;
    dtypes) for spec in "f32 reference 8" "f64 reference 8" "f16 reference 8" "bf16 reference 8" \
                        "i32 reference 8" "i64 reference 8" "u8 reference 8" "i8 reference 8" \
                        "f16 accum 8" "bf16 accum 8" "f32 reference 16" "bf16 reference 16" \
                        "f32 reference 2"; do
              set -- $spec
              run dt_$1_$2_$3 200 python bench.py --dtype $1 --mode $2 --workers $3 --steps 50 \
                  --no-cpu-baseline --no-scaling --no-cfg3 --no-fp16 --no-e2e || exit 1
            done ;;
    configs) run configs 900 python tools/bench_configs.py --only cfg1,sweep,cfg4,cfg5,cfg2e2e ;;
    pmc3)  run pmc_cfg3 400 python tools/pmc_cfg3.py "$OUT/pmc_cfg3" ;;
    cfg3prof) run cfg3_prof 300 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$OUT/cfg3prof" -o cfg3 -- ./tools/cfg3_native tools/cfg3_resnet50_table.txt 100 3 ;;
    cfg3py) run cfg3_python 600 python tools/bench_configs.py --only cfg3 ;;
    cfg1ab) run cfg1py_default 300 python tools/bench_configs.py --only cfg1 &&
            run cfg1py_d2hnormal 300 env BPSR_SERVER_D2H_PRIORITY=normal python tools/bench_configs.py --only cfg1 &&
            run cfg1py_memcpy 300 env BPSR_SERVER_PULL_COPY=memcpy python tools/bench_configs.py --only cfg1 &&
            run cfg1py_both 300 env BPSR_SERVER_PULL_COPY=memcpy BPSR_SERVER_D2H_PRIORITY=normal python tools/bench_configs.py --only cfg1 &&
            run cfg1py_default2 300 python tools/bench_configs.py --only cfg1 ;;
    cfg1pull) run cfg1py_kernel_a 300 python tools/bench_configs.py --only cfg1 &&
             run cfg1py_memcpy_a 300 env BPSR_SERVER_PULL_COPY=memcpy python tools/bench_configs.py --only cfg1 &&
             run cfg1py_kernel_b 300 python tools/bench_configs.py --only cfg1 &&
             run cfg1py_memcpy_b 300 env BPSR_SERVER_PULL_COPY=memcpy python tools/bench_configs.py --only cfg1 &&
             run cfg1n_kernel 300 ./tools/cfg1_native 4 20 &&
             run cfg1n_memcpy 300 env BPSR_SERVER_PULL_COPY=memcpy ./tools/cfg1_native 4 20 ;;
    srv3)  run server_cfg3 300 ./tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 4 &&
           run server_cfg3_l8 300 ./tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 8 ;;
    srv3trace) run srv3_trace 300 rocprofv3 --hip-runtime-trace --kernel-trace --stats --output-format csv \
             -d "$OUT/srv3trace" -o srv3 -- ./tools/server_cfg3_native tools/cfg3_resnet50_table.txt 10 4 2 ;;
    policy) run hbm_policy 300 env PROBE_POLICY=1 ./tools/hbm_probe2 256 ;;
    bqsweep) for v in 1 2 4; do for o in 1 2 3; do
               run bq_v${v}_o${o} 200 env BPSR_BQ_VPT=$v BPSR_BQ_GATE_OCC=$o ./tools/cfg3_native tools/cfg3_resnet50_table.txt 200 5 || exit 1
             done; done ;;
    native) run native 400 python -u -m pytest tests/test_native_gpu.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    cfg1n) run cfg1_native 300 ./tools/cfg1_native 4 20 ;;
    cfg1memcpy) run cfg1_native_memcpy 300 env BPSR_SERVER_PULL_COPY=memcpy ./tools/cfg1_native 4 20 ;;
    cfg1prio) run cfg1_native_d2h_normal 300 env BPSR_SERVER_D2H_PRIORITY=normal ./tools/cfg1_native 4 20 ;;
    cfg1q16) run cfg1_native_hwq16 300 env GPU_MAX_HW_QUEUES=16 BPSR_SERVER_D2H_PRIORITY=normal ./tools/cfg1_native 4 20 ;;
    cfg1q8) run cfg1_native_hwq8 300 env GPU_MAX_HW_QUEUES=8 ./tools/cfg1_native 4 20 ;;
    cfg1trace) run cfg1_trace 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
             -d "$OUT/cfg1trace" -o cfg1 -- ./tools/cfg1_native 4 6 ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$OUT/prof" -o bench -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-scaling --no-cfg3 --no-fp16 --no-e2e ;;
    skew)  for k in 4096 8192 16384 24576 49152 81920 1064960; do
             run skew_$k 200 python bench.py --steps 100 --no-cpu-baseline --no-scaling --no-cfg3 --no-fp16 --skew $k || exit 1
           done
           run skew_sep 200 python bench.py --steps 100 --no-cpu-baseline --no-scaling --no-cfg3 --no-fp16 --layout separate ;;
    pmc)   run pmc 900 python tools/pmc_traffic.py --out "$OUT/pmc" --session "$TAG" ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "done"

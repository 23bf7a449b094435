#!/bin/bash
# Round-3 GPU session steps.  Each GPU step has its own time limit; the script
# stops at the first step that ends in anything other than success or an
# ordinary test failure (fault, abort, segfault, timeout).
#   usage: tools/gpu_r03.sh <tag> <steps...>
set -u
TAG=${1:-r03}; shift || true
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

SRV="tools/server_cfg3_native tools/cfg3_resnet50_table.txt"
for s in $STEPS; do
  case $s in
    gputest) run gputest 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    bench5) run bench5 400 python bench.py --steps 20 --warmup 5 ;;
    srv) for v in 0 1 4; do run srv_v$v 300 $SRV 20 4 $v || exit 1; done ;;
    srvall) run srvall 400 $SRV 20 4 ;;
    srvprof) for v in 0 4; do
               run srvprof_v$v 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/srvprof_v$v -o run -- $SRV 10 4 $v || exit 1
             done ;;
    cfg3) run cfg3 300 tools/cfg3_native tools/cfg3_resnet50_table.txt 200 7 tools/cfg3_resnet50_tasks.txt ;;
    cfg3prof) run cfg3prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/cfg3prof -o run -- tools/cfg3_native tools/cfg3_resnet50_table.txt 200 3 "" blockq_live_release ;;
    benchprof) run benchprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/benchprof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  # keep what comes back small: traces compressed, databases dropped
  find "$OUT" -name '*.db' -delete
  find "$OUT" -name '*_trace.csv' -size +1M -exec gzip -f {} \;
done

#!/bin/bash
# One GPU-box session from a list of steps, each "<limit_s>:<name>:<command>":
# every step runs under its own time limit (timeout -k 10), its output goes
# to gpurun_out/<tag>/<name>.log, and the session stops at the first step that
# ends in anything but success or an ordinary failure (1): a fault, abort,
# segfault or time limit ends it there.
#   usage: tools/gpu_session.sh <tag> "300:tests:python -m pytest tests -m gpu -x -q" ...
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
for step in "$@"; do
  lim=${step%%:*}; rest=${step#*:}; name=${rest%%:*}; cmd=${rest#*:}
  echo "== $name ($(date +%T)) $cmd" | tee -a "$OUT/steps.log"
  timeout -k 10 "$lim" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -4 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)" | tee -a "$OUT/steps.log"
    exit $rc
  fi
done
echo "done"

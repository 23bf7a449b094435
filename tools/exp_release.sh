set -u
mkdir -p gpurun_out/r02s81
export TMPDIR=/tmp
for m in kernel copy kernel copy; do
  echo "== $m"
  BPSR_BQ_RELEASE=$m timeout -k 10 120 ./tools/cfg3_native tools/cfg3_resnet50_table.txt 200 5 "" blockq > gpurun_out/r02s81/cfg3_$m.log 2>&1 || { echo "rc=$?"; cat gpurun_out/r02s81/cfg3_$m.log; exit 1; }
  cat gpurun_out/r02s81/cfg3_$m.log | cut -c1-200
done

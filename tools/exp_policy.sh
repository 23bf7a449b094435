set -u
mkdir -p gpurun_out/r02s84
for mb in 66 256 66 256; do
  PROBE_POLICY=1 timeout -k 10 120 ./tools/hbm_probe2 $mb > gpurun_out/r02s84/pol_$mb.jsonl 2>&1 || { echo rc=$?; cat gpurun_out/r02s84/pol_$mb.jsonl; exit 1; }
  echo "== $mb"; grep '"rep": 1' gpurun_out/r02s84/pol_$mb.jsonl
done

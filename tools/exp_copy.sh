set -u
O=gpurun_out/r02s91
mkdir -p $O
for r in 1 2; do for w in 0 96; do
  BPSR_WT_MAX_MIB=$w timeout -k 10 200 python tools/copy_probe.py 1,4,16,33,64,128,256 > $O/copy_w${w}_r$r.jsonl 2> $O/copy_w${w}_r$r.err || { echo "rc=$?"; tail $O/copy_w${w}_r$r.err; exit 1; }
  echo "w=$w r=$r"; cat $O/copy_w${w}_r$r.jsonl
done; done

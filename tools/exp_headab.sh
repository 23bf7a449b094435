set -u
O=gpurun_out/r02s97
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do for t in A B; do
  d=.; x=--no-e2e; [ $t = A ] && d=r02ab && x=
  (cd $d && timeout -k 10 200 python bench.py --steps 200 --no-cpu-baseline --no-cfg3 --no-fp16 $x --no-scaling) > $O/b_$t$r.json 2>$O/b_$t$r.err || { echo "rc=$?"; tail $O/b_$t$r.err; exit 1; }
  python -c "import json; b=json.load(open('$O/b_$t$r.json')); print('$t$r', b['roofline']['kernel_ms'], b['ms_per_step'], b['check_vs_torch_fold'])"
done; done

export TMPDIR=/tmp; mkdir -p gpurun_out/r03s47
OUT=gpurun_out/r03s47
for v in 6 4; do for l in 1 4; do
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/tr_v${v}_l${l} -o run -- tools/server_cfg3_native tools/cfg3_resnet50_table.txt 20 $l $v > $OUT/srv_v${v}_l${l}.json 2>> $OUT/err.log || exit 1
done; done
find $OUT -name '*.db' -delete
for d in $OUT/tr_*; do echo "$d $(python tools/trace_gaps.py $d --window-ms 4 --min-us 10)"; done
cat $OUT/srv_*.json | cut -c1-400

# Diagnostic: grep insert phase stamps with hits in the map's flush order
# (default) vs sorted by position (--opt grep_sort_hits=1): does input locality
# (address translation) bound the insert?
set -e
out=gpurun_out/r5ay
mkdir -p $out
for o in 0 1 0 1; do
MRG_DEBUG_TIMES=1 timeout -k 10 300 python -u bench.py --workload c3 --steps 2 --warmup 1 --no-oracle --no-cpu-baseline --no-pcie --no-pipelined --splits 1 --opt grep_sort_hits=$o > $out/st_$o.json 2> $out/st_$o.err
echo sort_hits=$o; grep "grep insert" $out/st_$o.err | tail -1
python -c "import json;d=json.load(open('$out/st_$o.json'));print(d['value'],d['phases_ms'])"
done

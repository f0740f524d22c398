# grep reduce: radix over 16 key bytes (default) vs 8 (--opt grep_sort_k1=-1), C3.
set -e
out=gpurun_out/r5at
mkdir -p $out
for i in 1 2; do
for o in 0 -1; do
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu-baseline --no-pcie --no-pipelined --splits 2 --opt grep_sort_k1=$o > $out/c3_k1${o}_$i.json 2> $out/c3_k1${o}_$i.err
python -c "import json;d=json.load(open('$out/c3_k1${o}_$i.json'));print('k1=$o',d['value'],'reduce',d['phases_ms']['reduce'],d['checks'].get('exact_vs_oracle'))"
done
done

# Per-process aggregation time over 4 bench processes (the split's round-0
# aggregation is bimodal across processes: ~1.02 or ~1.24 ms), with the given options.
mkdir -p gpurun_out/aggm
for i in 1 2 3 4; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --steps 3 --warmup 1 "$@" > gpurun_out/aggm/b$i.json 2> gpurun_out/aggm/b$i.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/aggm/b$i.json'));print('run $i',d['value'],d['phases_ms']['map_kernel'],d['phases_ms']['agg'],d['spill_region_full_words'],d['checks']['total_words_match'])"
done

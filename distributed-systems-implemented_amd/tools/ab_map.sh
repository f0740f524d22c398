# A/B of library builds on the C2 bench (map kernel and end-to-end), alternating
# runs so box drift hits both: build/libmrgpu_base.so vs build/libmrgpu.so
set -e
mkdir -p gpurun_out/ab
B="python bench.py --no-cpu-baseline --no-pcie --steps 5"
L=distributed-systems-implemented_amd/build
for i in 1 2; do
for lib in base cur; do
  lp=$L/libmrgpu_$lib.so; [ $lib = cur ] && lp=$L/libmrgpu.so
  tag=${lib}_$i
  MRGPU_LIB=$lp timeout -k 10 200 $B "$@" > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err
  python -c "import json;d=json.load(open('gpurun_out/ab/$tag.json'));print('$tag',d['value'],d['phases_ms']['map_kernel'],d['phases_ms']['agg'],d['checks'].get('total_words_match'))"
done
done

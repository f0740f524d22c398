set -e
mkdir -p gpurun_out/ab
B="python bench.py --no-cpu-baseline --no-pcie --steps 5"
L=distributed-systems-implemented_amd/build
for v in "cur:" "nowb:" "nowb:--opt map_mode=32" "nowb:--opt map_mode=16" "cur:--opt map_mode=32" "nowb:--opt spill_buckets=512"; do
  lib=${v%%:*}; opt=${v#*:}; tag=$(echo "$lib$opt" | tr -c 'a-z0-9' '_')
  lp=$L/libmrgpu_$lib.so; [ $lib = cur ] && lp=$L/libmrgpu.so
  MRGPU_LIB=$lp timeout -k 10 200 $B $opt > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err
  python -c "import json;d=json.load(open('gpurun_out/ab/$tag.json'));print('$tag',d['value'],d['phases_ms']['map_kernel'],d['phases_ms']['agg'])"
done

# A/B of library variants (build/libmrgpu_<name>.so) on bench.py workloads,
# alternating variants twice so box drift hits all:
#   bash tools/ab_libs.sh OUT "c2 c5" name1 name2 ...
set -e
out=gpurun_out/${1:?}; shift
wls=$1; shift
mkdir -p $out
L=distributed-systems-implemented_amd/build
for i in 1 2; do
for w in $wls; do
for v in "$@"; do
  extra=""
  [ $w = c5 ] && extra="--files 40 --steps 3 --warmup 2"
  MRGPU_LIB=$L/libmrgpu_$v.so timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-pcie --no-oracle --no-pipelined --splits 2 $extra > $out/${w}_${v}_$i.json 2> $out/${w}_${v}_$i.err
  python -c "import json;d=json.load(open('$out/${w}_${v}_$i.json'));print('$w $v $i',d['value'],'map',d['phases_ms']['map_kernel'],'agg',d['phases_ms']['agg'],d['checks'].get('total_words_match'))"
done
done
done

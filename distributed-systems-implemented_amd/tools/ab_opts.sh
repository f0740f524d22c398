# A/B of library options on bench workloads, alternating so box drift hits all:
#   bash tools/ab_opts.sh OUT "c2 c5" "optA" "optB" ...   (an opt string: "" or "--opt name=v --opt ...")
set -e
out=gpurun_out/${1:?}; shift
wls=$1; shift
mkdir -p $out
for i in 1 2; do
for w in $wls; do
k=0
for o in "$@"; do
  k=$((k+1))
  extra=""
  [ $w = c5 ] && extra="--steps 3 --warmup 1"
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-pcie --no-oracle $extra $o > $out/${w}_${k}_$i.json 2> $out/${w}_${k}_$i.err
  python -c "import json;d=json.load(open('$out/${w}_${k}_$i.json'));p=d['phases_ms'];print('$w [$o] $i',d['value'],'map',p['map_kernel'],'agg',p['agg'],'reduce',p['reduce'],'d2h',p['d2h'],'ms',d['ms_per_step'])"
done
done
done

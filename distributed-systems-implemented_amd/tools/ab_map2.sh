# A/B of library variants (build/libmrgpu_<name>.so) on the map kernel alone
# (tools/mapprobe.py, mode 0 = the exact kernel; min over reps), alternating the
# variants twice so box drift hits all of them:
#   bash tools/ab_map2.sh OUT WORKLOAD name1 name2 ...
set -e
out=gpurun_out/${1:?}; shift
wl=$1; shift
mkdir -p $out
L=distributed-systems-implemented_amd/build
for i in ${ROUNDS:-1 2}; do
for v in "$@"; do
  MRGPU_LIB=$L/libmrgpu_$v.so timeout -k 10 240 python distributed-systems-implemented_amd/tools/mapprobe.py --workload $wl --modes 0 --reps 5 > $out/${wl}_${v}_$i.jsonl 2> $out/${wl}_${v}_$i.err
  python -c "import json;d=json.loads(open('$out/${wl}_${v}_$i.jsonl').read().splitlines()[-1]);print('$wl $v $i map %.3f agg %.3f spilled %d hits %d all %s' % (d['map_kernel_ms'], d['agg_ms'], d['spilled'], d['dict_hits'], d.get('all_ms')))"
done
done

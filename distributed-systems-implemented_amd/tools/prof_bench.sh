# rocprofv3 kernel-trace summary of one bench.py workload:
#   bash tools/prof_bench.sh OUT WORKLOAD [bench args...]
set -e
out=gpurun_out/${1:?}; shift
w=${1:?}; shift
mkdir -p $out
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o $w -- python3 bench.py --workload $w --no-cpu-baseline --no-pcie --no-oracle --steps 5 "$@" > $out/${w}_prof.json 2> $out/${w}_prof.err
f=$(find $out/prof -name "*.db" | head -1)
python3 distributed-systems-implemented_amd/tools/prof_summary.py "$f" $out/${w}_kernels.csv > /dev/null
head -16 $out/${w}_kernels.csv
rm -rf $out/prof  # the trace database (tens of MB): gpurun copies back at most 64 MiB

# Diagnostic: does the output's edge-byte traffic (byte stores into pinned host
# memory at each 128-line block's two partial 16-byte words) cost the grep
# formatting kernel time?  ne = those stores skipped (timing only: the output
# is wrong there), against the default library, kernel trace of each.
set -e
out=gpurun_out/r5ba
mkdir -p $out
L=distributed-systems-implemented_amd/build
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in main ne; do
lib=$L/libmrgpu.so; [ $v = ne ] && lib=$L/libmrgpu_ne.so
MRGPU_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_$v -o c3 -- python3 bench.py --workload c3 --steps 4 --warmup 1 --no-oracle --no-cpu-baseline --no-pcie --no-pipelined --splits 1 > $out/$v.json 2> $out/$v.err || echo "($v: exit $?)"
f=$(find $out/prof_$v -name "*.db" | head -1)
python3 distributed-systems-implemented_amd/tools/prof_summary.py "$f" $out/${v}_kernels.csv > /dev/null
echo $v; grep -E "write_lines|grep_map" $out/${v}_kernels.csv
rm -rf $out/prof_$v
done

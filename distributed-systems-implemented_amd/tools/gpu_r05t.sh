set -e
mkdir -p gpurun_out/r5t
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/r5t/prof -o c3 -- python3 $R/bench.py --workload c3 --no-cpu-baseline --no-pcie --no-oracle --no-pipelined --steps 3 --warmup 1 > $R/gpurun_out/r5t/c3.json 2> $R/gpurun_out/r5t/c3.err
cd $R
f=$(find gpurun_out/r5t/prof -name "*.db" | head -1)
python3 distributed-systems-implemented_amd/tools/timeline.py "$f" grep_map_kernel -2 > gpurun_out/r5t/timeline.txt
python3 distributed-systems-implemented_amd/tools/timeline.py "$f" grep_map_kernel -1 >> gpurun_out/r5t/timeline.txt
rm -rf gpurun_out/r5t/prof

set -e
mkdir -p gpurun_out/r5u
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_coordinator.py -m gpu -x -q --timeout 120 --timeout-method thread -k "grep or job or coordinator" > gpurun_out/r5u/tests.log 2>&1
B="python3 bench.py --workload c3 --no-cpu-baseline --no-pcie --no-pipelined --steps 5 --warmup 2"
for i in 1 2; do
timeout -k 10 300 $B > gpurun_out/r5u/new_$i.json 2> gpurun_out/r5u/new_$i.err
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/r5u/prof -o c3 -- python3 $R/bench.py --workload c3 --no-cpu-baseline --no-pcie --no-oracle --no-pipelined --steps 3 --warmup 1 > $R/gpurun_out/r5u/c3prof.json 2> $R/gpurun_out/r5u/c3prof.err
cd $R
f=$(find gpurun_out/r5u/prof -name "*.db" | head -1)
python3 distributed-systems-implemented_amd/tools/timeline.py "$f" grep_map_kernel -2 > gpurun_out/r5u/timeline.txt
rm -rf gpurun_out/r5u/prof

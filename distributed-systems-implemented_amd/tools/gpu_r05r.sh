set -e
mkdir -p gpurun_out/r5r
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "grep or job" > gpurun_out/r5r/tests.log 2>&1
B="python3 bench.py --workload c3 --no-cpu-baseline --no-pcie --no-oracle --no-pipelined --steps 5 --warmup 2"
for i in 1 2; do
timeout -k 10 300 $B --opt grep_sort_hits=1 > gpurun_out/r5r/base_$i.json 2> gpurun_out/r5r/base_$i.err
timeout -k 10 300 $B > gpurun_out/r5r/uns_$i.json 2> gpurun_out/r5r/uns_$i.err
timeout -k 10 300 $B --opt out_direct=2 > gpurun_out/r5r/dir_$i.json 2> gpurun_out/r5r/dir_$i.err
done
timeout -k 10 500 bash distributed-systems-implemented_amd/tools/prof_bench.sh r5r/c5 c5 --steps 2 --warmup 1 > gpurun_out/r5r/c5prof.log 2>&1

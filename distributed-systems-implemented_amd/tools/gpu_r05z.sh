set -e
mkdir -p gpurun_out/r5z
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "grep or tied or sort or reduce" > gpurun_out/r5z/tests.log 2>&1
for i in 1 2 3; do
timeout -k 10 300 python3 bench.py --workload c3 --no-cpu-baseline --no-pcie --no-pipelined --steps 5 --warmup 2 > gpurun_out/r5z/c3_$i.json 2> gpurun_out/r5z/c3_$i.err
done
MRG_DEBUG_TIES=1 timeout -k 10 300 python3 bench.py --workload c3 --no-cpu-baseline --no-pcie --no-pipelined --no-oracle --steps 2 --warmup 1 > gpurun_out/r5z/c3_ties.json 2> gpurun_out/r5z/c3_ties.err

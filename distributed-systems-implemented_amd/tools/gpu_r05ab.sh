set -e
mkdir -p gpurun_out/r5ac
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_coordinator.py -m gpu -x -q --timeout 200 --timeout-method thread -k "grep or job or coordinator or export" > gpurun_out/r5ac/tests.log 2>&1
for i in 1 2 3; do
timeout -k 10 300 python3 bench.py --workload c3 --no-cpu-baseline --no-pcie --no-pipelined --steps 5 --warmup 2 > gpurun_out/r5ac/c3_$i.json 2> gpurun_out/r5ac/c3_$i.err
done

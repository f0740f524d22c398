set -e
mkdir -p gpurun_out/r5v
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "grep or job" > gpurun_out/r5v/tests.log 2>&1
MRG_DEBUG_TIES=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -s --timeout 120 --timeout-method thread -k "log_prefix" > gpurun_out/r5v/ties.log 2>&1
B="python3 bench.py --workload c3 --no-cpu-baseline --no-pcie --no-pipelined --steps 5 --warmup 2"
for i in 1 2; do
timeout -k 10 300 $B > gpurun_out/r5v/new_$i.json 2> gpurun_out/r5v/new_$i.err
done

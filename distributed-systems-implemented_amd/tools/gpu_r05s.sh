set -e
mkdir -p gpurun_out/r5s
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5s/tests.log 2>&1
B="python3 bench.py --workload c3 --no-cpu-baseline --no-pcie --no-pipelined --steps 5 --warmup 2"
for i in 1 2; do
timeout -k 10 300 $B --no-oracle --opt grep_emit=0 > gpurun_out/r5s/old_$i.json 2> gpurun_out/r5s/old_$i.err
timeout -k 10 300 $B > gpurun_out/r5s/new_$i.json 2> gpurun_out/r5s/new_$i.err
done

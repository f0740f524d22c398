set -e
mkdir -p gpurun_out/r5y
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "radix or sort or reduce or grep or tied" > gpurun_out/r5y/tests.log 2>&1
for i in 1 2; do
for v in d8 d10; do
MRGPU_LIB=$R/distributed-systems-implemented_amd/build/libmrgpu_$v.so timeout -k 10 300 python3 bench.py --workload c3 --no-cpu-baseline --no-pcie --no-pipelined --no-oracle --steps 5 --warmup 2 > gpurun_out/r5y/c3_${v}_$i.json 2> gpurun_out/r5y/c3_${v}_$i.err
MRGPU_LIB=$R/distributed-systems-implemented_amd/build/libmrgpu_$v.so timeout -k 10 300 python3 bench.py --workload c2 --no-cpu-baseline --no-pcie --no-pipelined --no-oracle --steps 5 --warmup 2 > gpurun_out/r5y/c2_${v}_$i.json 2> gpurun_out/r5y/c2_${v}_$i.err
done
done

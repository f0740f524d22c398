set -e
mkdir -p gpurun_out/r5ah
R=$GRAFT_REPO_ROOT
MRGPU_LIB=$R/distributed-systems-implemented_amd/build/libmrgpu_nl4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_coordinator.py -m gpu -x -q --timeout 200 --timeout-method thread -k "grep or job or coordinator" > gpurun_out/r5ah/tests.log 2>&1
for i in 1 2; do
for v in head nl4; do
MRGPU_LIB=$R/distributed-systems-implemented_amd/build/libmrgpu_$v.so timeout -k 10 300 python3 bench.py --workload c3 --no-cpu-baseline --no-pcie --no-pipelined --no-oracle --steps 5 --warmup 2 > gpurun_out/r5ah/c3_${v}_$i.json 2> gpurun_out/r5ah/c3_${v}_$i.err
done
done

set -e
mkdir -p gpurun_out/r5w
R=$GRAFT_REPO_ROOT
for i in 1 2; do
for v in cur rows2; do
MRGPU_LIB=$R/distributed-systems-implemented_amd/build/libmrgpu_$v.so timeout -k 10 300 python3 bench.py --workload c3 --no-cpu-baseline --no-pcie --no-pipelined --no-oracle --steps 5 --warmup 2 > gpurun_out/r5w/c3_${v}_$i.json 2> gpurun_out/r5w/c3_${v}_$i.err
MRGPU_LIB=$R/distributed-systems-implemented_amd/build/libmrgpu_$v.so timeout -k 10 300 python3 bench.py --workload c2 --no-cpu-baseline --no-pcie --no-pipelined --no-oracle --steps 5 --warmup 2 > gpurun_out/r5w/c2_${v}_$i.json 2> gpurun_out/r5w/c2_${v}_$i.err
done
done

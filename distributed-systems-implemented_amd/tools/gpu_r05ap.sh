# grep insert occupancy A/B (__launch_bounds__ min waves per SIMD 4 / 6 / 8):
# grep tests with the 8-wave build, phase stamps, C3 lines alternating.
set -e
out=gpurun_out/r5ap
mkdir -p $out
L=distributed-systems-implemented_amd/build
for v in w6 w8; do
MRGPU_LIB=$L/libmrgpu_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k grep > $out/tests_$v.log 2>&1
tail -1 $out/tests_$v.log
done
for v in w4 w6 w8; do
MRGPU_LIB=$L/libmrgpu_$v.so MRG_DEBUG_TIMES=1 timeout -k 10 300 python -u bench.py --workload c3 --steps 2 --warmup 1 --no-oracle --no-cpu-baseline --no-pcie --no-pipelined --splits 1 > $out/st_$v.json 2> $out/st_$v.err
echo $v; grep "grep insert" $out/st_$v.err | tail -1
done
timeout -k 10 900 bash distributed-systems-implemented_amd/tools/ab_libs.sh r5ap c3 w4 w6 w8

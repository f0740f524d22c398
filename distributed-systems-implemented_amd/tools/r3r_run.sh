set -e
out=gpurun_out/r3r
mkdir -p $out
MRG_DEBUG_TIES=1 timeout -k 10 300 python -u bench.py --workload c3 --no-cpu-baseline --no-pcie --no-oracle --steps 2 --warmup 1 > $out/dbg.json 2> $out/dbg.err
grep "\[ties\]" $out/dbg.err | tail -3
MRGPU_LIB=distributed-systems-implemented_amd/build/libmrgpu_r4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "radix_sort_hook or sort_variants" > $out/r4_tests.log 2>&1
tail -1 $out/r4_tests.log
bash distributed-systems-implemented_amd/tools/ab_libs.sh r3r/ab "c3 c2" base cur r4

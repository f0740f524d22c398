set -e
mkdir -p gpurun_out/r5h
MRGPU_LIB=distributed-systems-implemented_amd/build/libmrgpu_d1p.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wc and not exchange_group_c" > gpurun_out/r5h/tests_d1p.log 2>&1
ROUNDS="1 2" bash distributed-systems-implemented_amd/tools/ab_map2.sh r5h c2 base basep d1 d1p

set -e
mkdir -p gpurun_out/r5f
MRGPU_LIB=distributed-systems-implemented_amd/build/libmrgpu_d1m.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wc and not exchange_group_c" > gpurun_out/r5f/tests_d1m.log 2>&1
bash distributed-systems-implemented_amd/tools/ab_map2.sh r5f c2 base basem d1 d1m

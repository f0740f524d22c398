set -e
mkdir -p gpurun_out/r5i
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "long or utf8 or lean or synthetic or edge or staged or spill" > gpurun_out/r5i/tests.log 2>&1
ROUNDS="1 2" bash distributed-systems-implemented_amd/tools/ab_map2.sh r5i c2u old new
ROUNDS="1" bash distributed-systems-implemented_amd/tools/ab_map2.sh r5i c2 old new

set -e
mkdir -p gpurun_out/r3i
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "high_cardinality or aggregator_overflow or c5_shape or wc_large or edge" > gpurun_out/r3i/gpu_tests.log 2>&1
tail -1 gpurun_out/r3i/gpu_tests.log
SKIP_TESTS=1 bash distributed-systems-implemented_amd/tools/ab_run.sh r3i "c5" cur nodrain nostage2

set -e
mkdir -p gpurun_out/r3m
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3m/gpu_tests.log 2>&1
tail -1 gpurun_out/r3m/gpu_tests.log
SKIP_TESTS=1 bash distributed-systems-implemented_amd/tools/ab_run.sh r3m "c2 c2u" base cur

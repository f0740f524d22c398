set -e
mkdir -p gpurun_out/r3l
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3l/gpu_tests.log 2>&1
tail -1 gpurun_out/r3l/gpu_tests.log
SKIP_TESTS=1 bash distributed-systems-implemented_amd/tools/ab_run.sh r3l "c2u c2" cur
bash distributed-systems-implemented_amd/tools/prof_bench.sh r3l/prof c2

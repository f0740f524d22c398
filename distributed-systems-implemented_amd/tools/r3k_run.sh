set -e
mkdir -p gpurun_out/r3k
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3k/gpu_tests.log 2>&1
tail -1 gpurun_out/r3k/gpu_tests.log
SKIP_TESTS=1 bash distributed-systems-implemented_amd/tools/ab_run.sh r3k "c2u c3" cur
bash distributed-systems-implemented_amd/tools/prof_bench.sh r3k/prof c3

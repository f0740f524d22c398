set -e
mkdir -p gpurun_out/r3e
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "sort or bucketed or large" > gpurun_out/r3e/sort_tests.log 2>&1
tail -1 gpurun_out/r3e/sort_tests.log
bash distributed-systems-implemented_amd/tools/ab_opts.sh r3e/ab "c2 c5" "" "--opt sort_prefix32=0"

set -e
mkdir -p gpurun_out/r3h
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3h/gpu_tests.log 2>&1
tail -1 gpurun_out/r3h/gpu_tests.log
bash distributed-systems-implemented_amd/tools/ab_opts.sh r3h/ab "c2 c3" "" "--opt out_direct=-1"

set -e
mkdir -p gpurun_out/r5a
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5a/gpu_tests.log 2>&1
timeout -k 10 300 python -u distributed-systems-implemented_amd/tools/mapprobe.py --modes 1,2,4,16,32,0 --reps 3 > gpurun_out/r5a/mapprobe_c2.jsonl 2> gpurun_out/r5a/mapprobe_c2.err

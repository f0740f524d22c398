set -e
mkdir -p gpurun_out/r3f
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3f/gpu_tests.log 2>&1
tail -1 gpurun_out/r3f/gpu_tests.log
for nb in 256; do
timeout -k 10 300 python -u distributed-systems-implemented_amd/tools/mapprobe.py --workload c5 --modes 2,4,16,32,0 --reps 2 --opt spill_buckets=$nb > gpurun_out/r3f/c5_modes_nb$nb.json 2> gpurun_out/r3f/c5_modes_nb$nb.err
cat gpurun_out/r3f/c5_modes_nb$nb.json
done
timeout -k 10 300 python -u distributed-systems-implemented_amd/tools/mapprobe.py --workload c5 --modes 0 --reps 2 --opt spill_buckets=2048 > gpurun_out/r3f/c5_nb2048.json 2> gpurun_out/r3f/c5_nb2048.err
cat gpurun_out/r3f/c5_nb2048.json
SKIP_TESTS=1 bash distributed-systems-implemented_amd/tools/ab_run.sh r3f "c5" base cur

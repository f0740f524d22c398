set -e
mkdir -p gpurun_out/r5c
for v in base d1; do
MRG_DEBUG_TIMES=1 MRGPU_LIB=distributed-systems-implemented_amd/build/libmrgpu_$v.so timeout -k 10 200 python distributed-systems-implemented_amd/tools/mapprobe.py --modes 0 --reps 3 > gpurun_out/r5c/$v.jsonl 2> gpurun_out/r5c/$v.err
done
MRG_DEBUG_TIES=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "tied_runs or log_prefix or radix_sort_hook or long_tie" > gpurun_out/r5c/ties.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "c5_p8" > gpurun_out/r5c/p8.log 2>&1
timeout -k 10 400 python -u bench.py --group-rehearsal > gpurun_out/r5c/group.json 2> gpurun_out/r5c/group.err

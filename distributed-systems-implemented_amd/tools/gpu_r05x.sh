set -e
mkdir -p gpurun_out/r5x
R=$GRAFT_REPO_ROOT
MRGPU_LIB=$R/distributed-systems-implemented_amd/build/libmrgpu_w2.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wc and not grep" > gpurun_out/r5x/tests_w2.log 2>&1
for i in 1 2; do
for v in w4 w2; do
MRGPU_LIB=$R/distributed-systems-implemented_amd/build/libmrgpu_$v.so timeout -k 10 300 python3 distributed-systems-implemented_amd/tools/mapprobe.py --workload c5 --gb 10 --modes 0 --reps 3 > gpurun_out/r5x/c5_${v}_$i.jsonl 2> gpurun_out/r5x/c5_${v}_$i.err
MRGPU_LIB=$R/distributed-systems-implemented_amd/build/libmrgpu_$v.so timeout -k 10 300 python3 distributed-systems-implemented_amd/tools/mapprobe.py --workload c2 --modes 0 --reps 3 > gpurun_out/r5x/c2_${v}_$i.jsonl 2> gpurun_out/r5x/c2_${v}_$i.err
done
done

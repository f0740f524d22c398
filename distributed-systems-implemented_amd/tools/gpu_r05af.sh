set -e
mkdir -p gpurun_out/r5af
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "long or utf8 or lean or synthetic or edge or wc" > gpurun_out/r5af/tests.log 2>&1
for i in 1 2; do
for v in head el split; do
MRGPU_LIB=$R/distributed-systems-implemented_amd/build/libmrgpu_$v.so timeout -k 10 300 python3 distributed-systems-implemented_amd/tools/mapprobe.py --workload c2u --modes 0 --reps 4 > gpurun_out/r5af/c2u_${v}_$i.jsonl 2> gpurun_out/r5af/c2u_${v}_$i.err
done
MRGPU_LIB=$R/distributed-systems-implemented_amd/build/libmrgpu_split.so timeout -k 10 300 python3 distributed-systems-implemented_amd/tools/mapprobe.py --workload c2 --modes 0 --reps 4 > gpurun_out/r5af/c2_split_$i.jsonl 2> gpurun_out/r5af/c2_split_$i.err
MRGPU_LIB=$R/distributed-systems-implemented_amd/build/libmrgpu_head.so timeout -k 10 300 python3 distributed-systems-implemented_amd/tools/mapprobe.py --workload c2 --modes 0 --reps 4 > gpurun_out/r5af/c2_head_$i.jsonl 2> gpurun_out/r5af/c2_head_$i.err
done

set -e
mkdir -p gpurun_out/r5ad
R=$GRAFT_REPO_ROOT
MRGPU_LIB=$R/distributed-systems-implemented_amd/build/libmrgpu_km.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "long or utf8 or lean or synthetic or edge" > gpurun_out/r5ad/tests.log 2>&1
for i in 1 2; do
for v in head km; do
MRGPU_LIB=$R/distributed-systems-implemented_amd/build/libmrgpu_$v.so timeout -k 10 300 python3 distributed-systems-implemented_amd/tools/mapprobe.py --workload c2u --modes 0 --reps 4 > gpurun_out/r5ad/c2u_${v}_$i.jsonl 2> gpurun_out/r5ad/c2u_${v}_$i.err
MRGPU_LIB=$R/distributed-systems-implemented_amd/build/libmrgpu_$v.so timeout -k 10 300 python3 distributed-systems-implemented_amd/tools/mapprobe.py --workload c2 --modes 0 --reps 4 > gpurun_out/r5ad/c2_${v}_$i.jsonl 2> gpurun_out/r5ad/c2_${v}_$i.err
done
done

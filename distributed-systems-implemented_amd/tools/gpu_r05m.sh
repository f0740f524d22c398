set -e
mkdir -p gpurun_out/r5m
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "long or utf8 or lean or synthetic or edge" > gpurun_out/r5m/tests.log 2>&1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in b2 b4; do
MRG_DEBUG_TIMES=1 MRGPU_LIB=$R/distributed-systems-implemented_amd/build/libmrgpu_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5m/prof_$v -o c2u -- python3 $R/distributed-systems-implemented_amd/tools/mapprobe.py --workload c2u --modes 0 --reps 3 > $R/gpurun_out/r5m/$v.jsonl 2> $R/gpurun_out/r5m/$v.err
done

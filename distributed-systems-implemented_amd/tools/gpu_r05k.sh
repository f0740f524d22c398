set -e
mkdir -p gpurun_out/r5k
#timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "long or utf8 or lean or synthetic or edge" > gpurun_out/r5k/tests.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in abl2 abl4 new; do
MRG_DEBUG_TIMES=1 MRGPU_LIB=distributed-systems-implemented_amd/build/libmrgpu_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5k/prof_$v -o c2u -- python3 distributed-systems-implemented_amd/tools/mapprobe.py --workload c2u --modes 0 --reps 3 > gpurun_out/r5k/$v.jsonl 2> gpurun_out/r5k/$v.err
done

set -e
mkdir -p gpurun_out/r5p
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5p/tests.log 2>&1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in b2; do
MRG_DEBUG_TIMES=1 MRGPU_LIB=$R/distributed-systems-implemented_amd/build/libmrgpu_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5p/prof_$v -o c2u -- python3 $R/distributed-systems-implemented_amd/tools/mapprobe.py --workload c2u --modes 0 --reps 3 > $R/gpurun_out/r5p/$v.jsonl 2> $R/gpurun_out/r5p/$v.err
done

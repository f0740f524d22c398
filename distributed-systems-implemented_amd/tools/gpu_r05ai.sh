set -e
mkdir -p gpurun_out/r5ai
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in base s1k g1k g1ks1k; do
MRGPU_LIB=$R/distributed-systems-implemented_amd/build/libmrgpu_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5ai/prof_$v -o c2u -- python3 $R/distributed-systems-implemented_amd/tools/mapprobe.py --workload c2u --modes 0 --reps 3 > $R/gpurun_out/r5ai/$v.jsonl 2> $R/gpurun_out/r5ai/$v.err
done
cd $R
for v in base s1k g1k g1ks1k; do
MRGPU_LIB=$R/distributed-systems-implemented_amd/build/libmrgpu_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "long_words or long_records" > gpurun_out/r5ai/tests_$v.log 2>&1
done

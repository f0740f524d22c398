# grep insert: claim CAS as the first probe (c1) against load-then-CAS (c0):
# grep / coordinator GPU tests, insert phase stamps, C3 lines alternating.
set -e
out=gpurun_out/r5aq
mkdir -p $out
L=distributed-systems-implemented_amd/build
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "grep or smoke or coordinator or hosts or run_job or long" > $out/tests.log 2>&1
tail -1 $out/tests.log
for v in c0 c1; do
MRGPU_LIB=$L/libmrgpu_$v.so MRG_DEBUG_TIMES=1 timeout -k 10 300 python -u bench.py --workload c3 --steps 2 --warmup 1 --no-oracle --no-cpu-baseline --no-pcie --no-pipelined --splits 1 > $out/st_$v.json 2> $out/st_$v.err
echo $v; grep "grep insert" $out/st_$v.err | tail -1
done
timeout -k 10 900 bash distributed-systems-implemented_amd/tools/ab_libs.sh r5aq c3 c0 c1

# grep insert phase stamps (MRG_DEBUG_TIMES) on C3.
set -e
out=gpurun_out/r5ao
mkdir -p $out
MRG_DEBUG_TIMES=1 timeout -k 10 300 python -u bench.py --workload c3 --steps 2 --warmup 1 --no-oracle --no-cpu-baseline --no-pcie --no-pipelined --splits 1 > $out/c3.json 2> $out/c3.err
grep "grep insert" $out/c3.err | tail -4

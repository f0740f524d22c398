# Diagnostic: grep insert phase stamps with the claim's count atomic replaced by
# a (racy) load + store (nd) against the default library: is the insert bound
# by device atomics?  Timing only (counts may race; checks may report it).
set -e
out=gpurun_out/r5ax
mkdir -p $out
L=distributed-systems-implemented_amd/build
for v in main nd main nd; do
lib=$L/libmrgpu.so; [ $v = nd ] && lib=$L/libmrgpu_nd.so
MRGPU_LIB=$lib MRG_DEBUG_TIMES=1 timeout -k 10 300 python -u bench.py --workload c3 --steps 2 --warmup 1 --no-oracle --no-cpu-baseline --no-pcie --no-pipelined --splits 1 > $out/st_$v.json 2> $out/st_$v.err || echo "($v: bench exit $?)"
echo $v; grep "grep insert" $out/st_$v.err | tail -1
done

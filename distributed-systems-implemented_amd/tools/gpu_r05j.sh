set -e
mkdir -p gpurun_out/r5j
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
MRG_DEBUG_TIMES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5j/prof -o c2u -- python3 distributed-systems-implemented_amd/tools/mapprobe.py --workload c2u --modes 0 --reps 2 > gpurun_out/r5j/probe.jsonl 2> gpurun_out/r5j/probe.err
f=$(find gpurun_out/r5j/prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r5j/kernel_stats.csv || true
rm -rf gpurun_out/r5j/prof/*/*.db 2>/dev/null || true

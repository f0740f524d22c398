set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_c5
cd /tmp && export TMPDIR=/tmp
for nb in 512 2048; do
for c in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pmc_c5/${nb}_$c -o p -- python3 $R/distributed-systems-implemented_amd/tools/mapprobe.py --workload c5 --gb 10 --modes 0 --reps 1 --opt spill_buckets=$nb > $R/gpurun_out/pmc_c5/${nb}_$c.log 2>&1
done
done

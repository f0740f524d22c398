# HBM traffic and instruction counters of the final C3 grep_map_kernel (round 5):
# short bench.py c3 run, each pass a run of its own (FETCH_SIZE and WRITE_SIZE
# cannot share one), plus the SQ instruction pass.
set -e
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r5bb
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
pass() {
    local name=$1; shift
    timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o p -- python3 $R/bench.py --workload c3 --no-cpu-baseline --no-pcie --no-oracle --steps 2 --warmup 1 > "$out/$name.log" 2>&1
}
pass p3 FETCH_SIZE
pass p4 WRITE_SIZE
pass p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS
cd $R
python3 distributed-systems-implemented_amd/tools/pmc_summary.py --each $out grep_map > $out/summary.txt
find $out -name "*_counter_collection.csv" -size +20M -delete

set -e
mkdir -p gpurun_out/r5ae
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python3 distributed-systems-implemented_amd/tools/mapprobe.py --workload c5 --gb 10 --modes 2,4,16,32,0 --reps 3 > gpurun_out/r5ae/c5modes.jsonl 2> gpurun_out/r5ae/c5modes.err
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/r5ae/pmc_c5 -o p -- python3 $R/distributed-systems-implemented_amd/tools/mapprobe.py --workload c5 --gb 10 --modes 0 --reps 2 > $R/gpurun_out/r5ae/pmc_c5.log 2>&1

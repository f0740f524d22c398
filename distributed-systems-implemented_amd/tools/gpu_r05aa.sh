set -e
mkdir -p gpurun_out/r5aa
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python3 distributed-systems-implemented_amd/tools/mapprobe.py --workload c2u --modes 2,4,16,32,0 --reps 3 > gpurun_out/r5aa/modes.jsonl 2> gpurun_out/r5aa/modes.err
MRGPU_LIB=$R/distributed-systems-implemented_amd/build/libmrgpu_nolrec.so timeout -k 10 300 python3 distributed-systems-implemented_amd/tools/mapprobe.py --workload c2u --modes 2,4,0 --reps 3 > gpurun_out/r5aa/nolrec.jsonl 2> gpurun_out/r5aa/nolrec.err
timeout -k 10 300 python3 distributed-systems-implemented_amd/tools/mapprobe.py --workload c2 --modes 2,4,16,32,0 --reps 3 > gpurun_out/r5aa/c2modes.jsonl 2> gpurun_out/r5aa/c2modes.err

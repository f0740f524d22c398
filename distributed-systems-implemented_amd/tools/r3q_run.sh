set -e
bash distributed-systems-implemented_amd/tools/prof_bench.sh r3q/rank c3
bash distributed-systems-implemented_amd/tools/prof_bench.sh r3q/merge c3 --opt tie_rank=0

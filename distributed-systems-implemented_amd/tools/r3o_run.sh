set -e
bash distributed-systems-implemented_amd/tools/prof_bench.sh r3o c3
bash distributed-systems-implemented_amd/tools/prof_bench.sh r3o c5 --files 40 --steps 3 --warmup 1
bash distributed-systems-implemented_amd/tools/prof_bench.sh r3o c2

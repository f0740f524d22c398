# Round-5 final set, part B: bench C4 share and C5, rocprofv3 kernel summaries
# of C2 / C3, counter passes (C2 and C2u map kernels: per-chunk instruction
# counts and HBM traffic).
set -e
out=gpurun_out/final5g
mkdir -p $out
timeout -k 10 400 python -u bench.py --workload c4 --no-cpu-baseline --no-pcie > $out/c4.json 2> $out/c4.err
timeout -k 10 600 python -u bench.py --workload c5 --no-cpu-baseline --no-pcie --steps 3 --warmup 1 > $out/c5.json 2> $out/c5.err
for w in c4 c5; do python -c "import json;d=json.loads(open('$out/$w.json').read().strip().splitlines()[-1]);print('$w',d['value'],d['ms_per_step'],d['roofline']['frac'],d['phases_ms'],d['checks'].get('exact_vs_oracle'))"; done
timeout -k 10 450 bash distributed-systems-implemented_amd/tools/prof_bench.sh final5g/c2 c2
timeout -k 10 450 bash distributed-systems-implemented_amd/tools/prof_bench.sh final5g/c3 c3
R=$GRAFT_REPO_ROOT
timeout -k 10 500 bash distributed-systems-implemented_amd/tools/pmc_passes.sh $R/$out/pmc_c2 --workload c2 --modes 0 --reps 2
timeout -k 10 500 bash distributed-systems-implemented_amd/tools/pmc_passes.sh $R/$out/pmc_c2u --workload c2u --modes 0 --reps 2

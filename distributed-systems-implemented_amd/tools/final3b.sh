# Round-3 final measurement set, part B: C4 share, C5 (oracle-checked), the
# rocprofv3 kernel-trace summary of C2, and PMC passes over C2's map kernel
# (VALU/SALU/LDS per chunk; FETCH_SIZE and WRITE_SIZE in separate passes).
set -e
out=gpurun_out/final3
mkdir -p $out
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline --no-pcie > $out/c4.json 2> $out/c4.err
timeout -k 10 400 python -u bench.py --workload c5 --no-cpu-baseline --no-pcie --steps 3 --warmup 1 > $out/c5.json 2> $out/c5.err
for w in c4 c5; do python -c "import json;d=json.load(open('$out/$w.json'));print('$w',d['value'],d['ms_per_step'],d['roofline']['frac'],d['phases_ms'],'exact',d['checks'].get('exact_vs_oracle'))"; done
bash distributed-systems-implemented_amd/tools/prof_bench.sh final3/prof c2
bash distributed-systems-implemented_amd/tools/pmc_passes.sh $out/pmc --modes 0 --reps 1
python3 distributed-systems-implemented_amd/tools/pmc_summary.py --each $out/pmc wc_map_kernel > $out/pmc_summary.json
head -60 $out/pmc_summary.json
bash distributed-systems-implemented_amd/tools/pmc_passes.sh $out/pmc_c5 --workload c5 --gb 10 --modes 0 --reps 1
python3 distributed-systems-implemented_amd/tools/pmc_summary.py --each $out/pmc_c5 wc_map_kernel > $out/pmc_c5_summary.json
head -60 $out/pmc_c5_summary.json
bash distributed-systems-implemented_amd/tools/ab_opts.sh final3/abo "c2u" "--opt own_sort=1" "--opt own_sort=0"

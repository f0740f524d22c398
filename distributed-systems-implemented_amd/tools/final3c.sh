# Round-3 final set, part C: PMC passes over C5's map kernel as the bench runs it
# (2048 spill buckets; mapprobe's C5 mode otherwise keeps the 256-bucket layout).
set -e
out=gpurun_out/final3
bash distributed-systems-implemented_amd/tools/pmc_passes.sh $out/pmc_c5_2048 --workload c5 --gb 10 --modes 0 --reps 1 --opt spill_buckets=2048
python3 distributed-systems-implemented_amd/tools/pmc_summary.py --each $out/pmc_c5_2048 wc_map_kernel > $out/pmc_c5_2048_summary.json
head -40 $out/pmc_c5_2048_summary.json

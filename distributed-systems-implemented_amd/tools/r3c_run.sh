# VALU issue-cost probe, then the C5 map kernel with 256 vs 2048 spill buckets
set -e
mkdir -p gpurun_out/r3c
timeout -k 10 120 distributed-systems-implemented_amd/tools/ubench/valu_probe > gpurun_out/r3c/valu_probe.txt 2>&1
cat gpurun_out/r3c/valu_probe.txt
for nb in 2048 256 512; do
timeout -k 10 300 python -u distributed-systems-implemented_amd/tools/mapprobe.py --workload c5 --modes 0 --reps 2 --opt spill_buckets=$nb > gpurun_out/r3c/c5_nb$nb.json 2> gpurun_out/r3c/c5_nb$nb.err
cat gpurun_out/r3c/c5_nb$nb.json
done

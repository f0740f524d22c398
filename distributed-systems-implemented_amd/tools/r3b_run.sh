set -e
mkdir -p gpurun_out/r3b
timeout -k 10 120 distributed-systems-implemented_amd/tools/ubench/valu_probe > gpurun_out/r3b/valu_probe.txt 2>&1
cat gpurun_out/r3b/valu_probe.txt
timeout -k 10 300 python -u bench.py --workload c3 --no-pcie > gpurun_out/r3b/c3.json 2> gpurun_out/r3b/c3.err
timeout -k 10 400 python -u bench.py --workload c5 --no-cpu-baseline --no-pcie --steps 3 --warmup 1 > gpurun_out/r3b/c5.json 2> gpurun_out/r3b/c5.err
bash distributed-systems-implemented_amd/tools/prof_bench.sh r3b/prof c2
for w in c3 c5; do python -c "import json;d=json.load(open('gpurun_out/r3b/$w.json'));print('$w',d['value'],d['ms_per_step'],d['roofline']['frac'],d['phases_ms'],d['checks'].get('exact_vs_oracle'))"; done

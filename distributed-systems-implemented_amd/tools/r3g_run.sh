set -e
mkdir -p gpurun_out/r3g
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3g/gpu_tests.log 2>&1
tail -1 gpurun_out/r3g/gpu_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie > gpurun_out/r3g/c2.json 2> gpurun_out/r3g/c2.err
python -c "import json;d=json.load(open('gpurun_out/r3g/c2.json'));print('c2',d['value'],d['ms_per_step'],d['phases_ms'],d['checks'].get('exact_vs_oracle'))"
timeout -k 10 120 distributed-systems-implemented_amd/tools/ubench/h2h_probe > gpurun_out/r3g/h2h_probe.txt 2>&1
cat gpurun_out/r3g/h2h_probe.txt

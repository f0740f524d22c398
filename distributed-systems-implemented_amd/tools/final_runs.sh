# Round-end measurement set: GPU tests, bench lines for C2 (default, with CPU
# baseline and PCIe-inclusive), C3, C4's per-GPU share, C5, and a rocprofv3
# kernel-trace summary of C2.  Each step has its own time limit; any failure ends it.
set -e
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1
tail -2 gpurun_out/final/gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/final/c2.json 2> gpurun_out/final/c2.err
timeout -k 10 300 python bench.py --workload c3 > gpurun_out/final/c3.json 2> gpurun_out/final/c3.err
timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline --no-pcie > gpurun_out/final/c4.json 2> gpurun_out/final/c4.err
timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --no-pcie --steps 3 --warmup 1 > gpurun_out/final/c5.json 2> gpurun_out/final/c5.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof -o c2 -- python3 bench.py --no-cpu-baseline --no-pcie --steps 5 > gpurun_out/final/c2_prof.json 2> gpurun_out/final/c2_prof.err
for w in c2 c3 c4 c5; do python -c "import json;d=json.load(open('gpurun_out/final/$w.json'));print('$w',d['value'],d['ms_per_step'],d['roofline']['frac'],d['phases_ms'])"; done

# Round-5 final set, part A: GPU suite, smoke, bench lines C2 (default: CPU
# baseline, PCIe-inclusive, oracle), C3, C2u.  Each step under its own limit.
set -e
out=gpurun_out/final5f
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
tail -2 $out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1
tail -1 $out/smoke.log
timeout -k 10 500 python -u bench.py > $out/c2.json 2> $out/c2.err
timeout -k 10 400 python -u bench.py --workload c3 > $out/c3.json 2> $out/c3.err
timeout -k 10 400 python -u bench.py --workload c2u --no-cpu-baseline --no-pcie > $out/c2u.json 2> $out/c2u.err
for w in c2 c3 c2u; do python -c "import json;d=json.loads(open('$out/$w.json').read().strip().splitlines()[-1]);print('$w',d['value'],d['ms_per_step'],d['roofline']['frac'],d['phases_ms'],d['checks'].get('exact_vs_oracle'))"; done
timeout -k 10 450 bash distributed-systems-implemented_amd/tools/prof_bench.sh final5f/prof c3

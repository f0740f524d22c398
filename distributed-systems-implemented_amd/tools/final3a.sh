# Round-3 final measurement set, part A: GPU tests, smoke, bench lines with the
# full-size oracle check for C2 (default: + CPU baseline + PCIe-inclusive), C2u, C3.
set -e
out=gpurun_out/final3
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
tail -1 $out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
tail -1 $out/smoke.log
timeout -k 10 400 python -u bench.py > $out/c2.json 2> $out/c2.err
timeout -k 10 300 python -u bench.py --workload c2u --no-cpu-baseline --no-pcie > $out/c2u.json 2> $out/c2u.err
timeout -k 10 300 python -u bench.py --workload c3 --no-pcie > $out/c3.json 2> $out/c3.err
for w in c2 c2u c3; do python -c "import json;d=json.load(open('$out/$w.json'));print('$w',d['value'],d['ms_per_step'],d['roofline']['frac'],d['phases_ms'],'exact',d['checks'].get('exact_vs_oracle'))"; done

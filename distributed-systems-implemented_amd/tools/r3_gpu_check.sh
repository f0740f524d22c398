# Round-3 GPU check: -m gpu tests, smoke(), the default bench (C2 with the
# full-size oracle check) and the mixed-UTF-8 wc bench (C2u).  Each step has its
# own time limit; the first failure ends the script.
set -e
out=gpurun_out/${1:-r3b}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
tail -2 $out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
tail -1 $out/smoke.log
timeout -k 10 500 python -u bench.py > $out/c2.json 2> $out/c2.err
timeout -k 10 400 python -u bench.py --workload c2u --no-cpu-baseline --no-pcie > $out/c2u.json 2> $out/c2u.err
for w in c2 c2u; do python -c "import json;d=json.load(open('$out/$w.json'));print('$w',d['value'],d['ms_per_step'],d['roofline']['frac'],d['phases_ms'],d['checks'].get('exact_vs_oracle'),d['checks'].get('oracle_s'),d['cold_split'])"; done

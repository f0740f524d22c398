# grep map 4-byte prefix filter: the grep GPU tests, then the C3 bench line.
set -e
out=gpurun_out/r5ak
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "grep or smoke or coordinator or hosts" > $out/tests.log 2>&1
tail -2 $out/tests.log
timeout -k 10 400 python -u bench.py --workload c3 --no-cpu-baseline --no-pcie > $out/c3.json 2> $out/c3.err
python -c "import json;d=json.loads(open('$out/c3.json').read().strip().splitlines()[-1]);print('c3',d['value'],d['ms_per_step'],d['roofline']['frac'],d['phases_ms'],d['same_split_value'],d['checks'].get('exact_vs_oracle'))"

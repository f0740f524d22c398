# grep map with the single-compare tail-chunk test: the grep GPU tests (tail
# cases for every n % 4 included) and one C3 line.
set -e
out=gpurun_out/r5aw
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "grep or smoke or run_job or coordinator" > $out/tests.log 2>&1
tail -1 $out/tests.log
timeout -k 10 400 python -u bench.py --workload c3 --no-cpu-baseline --no-pcie > $out/c3.json 2> $out/c3.err
python -c "import json;d=json.loads(open('$out/c3.json').read().strip().splitlines()[-1]);print('c3',d['value'],d['ms_per_step'],d['roofline']['frac'],d['phases_ms'],d['same_split_value'],d['checks'].get('exact_vs_oracle'))"

# GPU test suite, then bench lines for the workloads named on the command line
# (default: c2 c2u c5), each under its own time limit; the first failure ends it.
#   bash distributed-systems-implemented_amd/tools/bench_set.sh OUT [workload ...]
set -e
out=gpurun_out/${1:?out dir}
shift
mkdir -p $out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
  tail -2 $out/gpu_tests.log
fi
for w in ${@:-c2 c2u c5}; do
  extra="--no-cpu-baseline --no-pcie"
  steps=""
  if [ $w = c5 ]; then steps="--steps 3 --warmup 1"; fi
  timeout -k 10 500 python -u bench.py --workload $w $extra $steps ${BENCH_ARGS:-} > $out/$w.json 2> $out/$w.err
  python -c "import json;d=json.load(open('$out/$w.json'));print('$w',d['value'],d['ms_per_step'],d['roofline']['frac'],d['phases_ms'],'exact',d['checks'].get('exact_vs_oracle'))"
done

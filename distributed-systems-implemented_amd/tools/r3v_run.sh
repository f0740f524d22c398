set -e
out=gpurun_out/r3v
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tied_runs or grep_edge or run_job_output or sort_variants or wc_edge" > $out/sel_tests.log 2>&1
tail -1 $out/sel_tests.log
MRG_DEBUG_TIES=1 timeout -k 10 300 python -u bench.py --workload c3 --no-cpu-baseline --no-pcie --no-oracle --steps 2 --warmup 1 > $out/dbg.json 2> $out/dbg.err
grep "\[ties\]" $out/dbg.err | tail -2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
tail -1 $out/gpu_tests.log
bash distributed-systems-implemented_amd/tools/ab_libs.sh r3v/ab "c3 c2" base cur
bash distributed-systems-implemented_amd/tools/ab_opts.sh r3v/abo "c3" "--opt out_direct=1" "--opt out_direct=-1"

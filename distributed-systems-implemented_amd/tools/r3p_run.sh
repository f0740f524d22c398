set -e
out=gpurun_out/r3p
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tied_runs or radix_sort_hook or sort_variants or grep_edge" > $out/sort_tests.log 2>&1
tail -1 $out/sort_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
tail -1 $out/gpu_tests.log
bash distributed-systems-implemented_amd/tools/ab_libs.sh r3p/ab "c3 c2" base cur
bash distributed-systems-implemented_amd/tools/ab_opts.sh r3p/abo "c3" "--opt tie_rank=1" "--opt tie_rank=0"

# grep map prefix filter: 32-bit compares into lane masks (z1, default) vs the
# zero-byte test (z0): grep GPU tests, then C3 lines alternating.
set -e
out=gpurun_out/r5au
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "grep or smoke or run_job" > $out/tests.log 2>&1
tail -1 $out/tests.log
timeout -k 10 900 bash distributed-systems-implemented_amd/tools/ab_libs.sh r5au c3 z0 z1

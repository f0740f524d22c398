# grep map with the ring unrolled (u1: constant slot addresses) vs HEAD (u0):
# grep GPU tests, then C3 lines alternating.
set -e
out=gpurun_out/r5bc
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "grep or smoke or run_job or coordinator" > $out/tests.log 2>&1
tail -1 $out/tests.log
timeout -k 10 900 bash distributed-systems-implemented_amd/tools/ab_libs.sh r5bc c3 u0 u1

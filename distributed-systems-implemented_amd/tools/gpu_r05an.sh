# grep insert: FNV-1a-32-only line pass (table hash from it and the length) and
# two counter atomics per workgroup step: grep / coordinator GPU tests, then C3
# A/B against the previous commit, and a kernel trace of the new one.
set -e
out=gpurun_out/r5an
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "grep or smoke or coordinator or hosts or run_job" > $out/tests.log 2>&1
tail -1 $out/tests.log
timeout -k 10 900 bash distributed-systems-implemented_amd/tools/ab_libs.sh r5an c3 base new
timeout -k 10 450 bash distributed-systems-implemented_amd/tools/prof_bench.sh r5an/prof c3

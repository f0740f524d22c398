set -e
out=gpurun_out/r3u
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
tail -1 $out/gpu_tests.log
bash distributed-systems-implemented_amd/tools/ab_libs.sh r3u/ab "c3 c2" cur

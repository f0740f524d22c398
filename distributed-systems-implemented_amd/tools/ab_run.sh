# GPU tests on the current library, then an A/B of library variants on bench workloads:
#   bash tools/ab_run.sh OUT "c2 c2u" name1 name2 ...   (SKIP_TESTS=1 to skip the tests)
set -e
out=gpurun_out/${1:?}; shift
mkdir -p $out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
  tail -1 $out/gpu_tests.log
fi
bash distributed-systems-implemented_amd/tools/ab_libs.sh ${out#gpurun_out/}/ab "$@"

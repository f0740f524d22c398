# radix pass look-back window A/B (16 / 32 tiles' words per round trip):
# sort / reduce tests with the 32 build, then C2 and C3 lines alternating.
set -e
out=gpurun_out/r5as
mkdir -p $out
L=distributed-systems-implemented_amd/build
MRGPU_LIB=$L/libmrgpu_lw32.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "radix or reduce or sort or tied or grep_synthetic or high_card" > $out/tests_lw32.log 2>&1
tail -1 $out/tests_lw32.log
timeout -k 10 900 bash distributed-systems-implemented_amd/tools/ab_libs.sh r5as "c3 c2" lw16 lw32

# grep map ring depth A/B (2 / 3 / 4 LDS slots per wave; the deeper rings with smaller match buffers, so two workgroups still fit a CU):
# the deeper rings, then C3 bench lines alternating the variants.
set -e
out=gpurun_out/r5am
mkdir -p $out
L=distributed-systems-implemented_amd/build
for v in gs3b gs4b; do
MRGPU_LIB=$L/libmrgpu_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k grep > $out/tests_$v.log 2>&1
tail -1 $out/tests_$v.log
done
timeout -k 10 900 bash distributed-systems-implemented_amd/tools/ab_libs.sh r5am c3 gs2 gs3b gs4b

set -e
out=gpurun_out/r3t
mkdir -p $out
for v in w16r4 w8r8 w8r16; do
MRGPU_LIB=distributed-systems-implemented_amd/build/libmrgpu_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "radix_sort_hook" > $out/${v}_tests.log 2>&1
echo "$v $(tail -1 $out/${v}_tests.log)"
done
bash distributed-systems-implemented_amd/tools/ab_libs.sh r3t/ab "c3 c2" cur w16r4 w8r8 w8r16

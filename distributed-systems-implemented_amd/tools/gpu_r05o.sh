mkdir -p gpurun_out/r5o /tmp/nobkt
cp distributed-systems-implemented_amd/build/libmrgpu_nobkt.so /tmp/nobkt/libmrgpu.so
timeout -k 10 200 python -u distributed-systems-implemented_amd/tools/coorddiff.py 1 > gpurun_out/r5o/cur1.log 2>&1 || exit 1
LD_LIBRARY_PATH=/tmp/nobkt timeout -k 10 200 python -u distributed-systems-implemented_amd/tools/coorddiff.py 1 > gpurun_out/r5o/nobkt1.log 2>&1 || exit 1

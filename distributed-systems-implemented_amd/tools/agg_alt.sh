# Diagnostic: is the per-process aggregation time a property of the spill pool's
# placement?  Two bench processes with two spill pools alternating per split
# (option spill_alt_pools); MRG_DEBUG_TIMES prints every split's round times.
mkdir -p gpurun_out/aggalt
for i in 1 2 3 4 5; do
  MRG_DEBUG_TIMES=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --steps 6 --warmup 2 --opt spill_alt_pools=1 \
    > gpurun_out/aggalt/b$i.json 2> gpurun_out/aggalt/b$i.err || exit 1
  grep "round 0" gpurun_out/aggalt/b$i.err | awk '{print $5}' | tr '\n' ' '; echo
done

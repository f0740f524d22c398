#!/bin/bash
# Two rocprofv3 counter passes (separate runs, as MI355X_MICROARCH.md prescribes)
# over tools/mapprobe.py.  usage: tools/pmc_passes.sh <outdir> <mapprobe args...>
set -e
out=$1; shift
R=$(cd "$(dirname "$0")/../.." && pwd)
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d "$out/p1" -o p -- python3 "$R/distributed-systems-implemented_amd/tools/mapprobe.py" "$@" > "$out/p1.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d "$out/p2" -o p -- python3 "$R/distributed-systems-implemented_amd/tools/mapprobe.py" "$@" > "$out/p2.log" 2>&1

#!/bin/bash
# rocprofv3 counter passes over tools/mapprobe.py, each pass a run of its own
# (MI355X_MICROARCH.md: rocprofv3 does not split counters over passes; FETCH_SIZE
# and WRITE_SIZE cannot share a pass).
# usage: tools/pmc_passes.sh <outdir> <mapprobe args...>
# Summarize with: python tools/pmc_summary.py <outdir>/p1 ... (or the whole outdir)
set -e
out=$(realpath -m "$1"); shift
R=$(cd "$(dirname "$0")/../.." && pwd)
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
probe="$R/distributed-systems-implemented_amd/tools/mapprobe.py"
pass() {
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o p -- python3 "$probe" $PROBE_ARGS \
        > "$out/$name.log" 2>&1
}
PROBE_ARGS="$*"
pass p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS
pass p2 SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE
pass p3 FETCH_SIZE
pass p4 WRITE_SIZE

#!/bin/bash
# SQ/GRBM counter passes over one f16x3 ensemble layer (tools/h3_pmc.py), one pass per run.
# usage (GPU box): bash tools/h3_pmc.sh [layer]
set -o pipefail
L=${1:-3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/rocprof_counters.txt" 2>&1 || true
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d "$R/gpurun_out/h3pmc_$i" -o run --output-format csv -- \
    python "$R/tools/h3_pmc.py" run $L 40 > "$R/gpurun_out/h3pmc_$i.log" 2>&1 \
    || { echo "pass $i FAILED"; tail -5 "$R/gpurun_out/h3pmc_$i.log"; exit 1; }
done
cd "$R" && python tools/h3_pmc.py parse gpurun_out/h3pmc_1 gpurun_out/h3pmc_2

#!/bin/bash
# Counter passes (one per run) over whole forwards: the one-launch form vs the per-layer launches.
# usage (GPU box): bash tools/fwd_pmc.sh [lanes]
set -o pipefail
B=${1:-5120}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA SQ_INSTS_SALU"
P3="TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCP_PENDING_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES TCP_CACHE_MISS TCP_PERF_SEL_TOTAL_READ TCC_HIT TCC_MISS GRBM_GUI_ACTIVE"
for mode in fused layers; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d "$R/gpurun_out/fwdpmc_${mode}_$i" -o run --output-format csv -- \
      python "$R/tools/fwd_pmc.py" run $mode $B 20 > "$R/gpurun_out/fwdpmc_${mode}_$i.log" 2>&1 \
      || { echo "$mode pass $i FAILED"; tail -5 "$R/gpurun_out/fwdpmc_${mode}_$i.log"; exit 1; }
  done
done
cd "$R" && python tools/fwd_pmc.py parse gpurun_out/fwdpmc_fused_1 gpurun_out/fwdpmc_fused_2 gpurun_out/fwdpmc_fused_3 \
  gpurun_out/fwdpmc_layers_1 gpurun_out/fwdpmc_layers_2 gpurun_out/fwdpmc_layers_3

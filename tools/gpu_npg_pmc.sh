#!/bin/bash
# NPG pass kernel PMC passes (FVP / VPG / EVAL dispatches of tools/npg_phase.py time).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/npg_pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
LIB=$R/amp_extensions_amd/libamx_hip.so
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/p1 -o run -- python3 $R/tools/npg_phase.py time $LIB 40960 197 36 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_MFMA SQ_WAVES --output-format csv -d $O/p2 -o run -- python3 $R/tools/npg_phase.py time $LIB 40960 197 36 > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
ls -R $O | head -20

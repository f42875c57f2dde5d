#!/bin/bash
# r04j: NPG pass phase stamps (tools/npg_phase.py trace: fvp, fvp_cached, vpg, eval)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 200 python tools/npg_phase.py trace > gpurun_out/r04j_npg_trace.txt 2>&1 || { tail -20 gpurun_out/r04j_npg_trace.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04j_npg_trace.txt | cut -c1-400

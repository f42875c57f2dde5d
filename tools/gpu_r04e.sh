#!/bin/bash
# r04e: NPG pass with swizzled small tiles: its tests, the update time, the SQ counters
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_npg.py tests/test_gpu_gae.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r04e.log 2>&1 || { tail -30 gpurun_out/pytest_r04e.log; exit 1; }
tail -1 gpurun_out/pytest_r04e.log
timeout -k 10 200 python tools/npg_time.py > gpurun_out/r04e_npg_time.txt 2>&1 || { tail -20 gpurun_out/r04e_npg_time.txt; exit 1; }
tail -3 gpurun_out/r04e_npg_time.txt
timeout -k 10 200 python tools/npg_phase.py time amp_extensions_amd/libamx_hip.so 40960 197 36 > gpurun_out/r04e_npg_phase.txt 2>&1 || { tail -20 gpurun_out/r04e_npg_phase.txt; exit 1; }
tail -8 gpurun_out/r04e_npg_phase.txt
bash tools/gpu_npg_pmc.sh > gpurun_out/r04e_npg_pmc.log 2>&1 || { tail -10 gpurun_out/r04e_npg_pmc.log; exit 1; }
echo pmc ok

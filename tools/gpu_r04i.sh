#!/bin/bash
# r04i: the NPG theta-forward cache -- GPU NPG tests (cached FVP bit-identical to the uncached),
# the pass times (tools/npg_phase.py time: fvp / vpg / eval / fvp_cached) and the update time.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_npg.py tests/test_gpu_gae.py > gpurun_out/pytest_r04i.log 2>&1 || { tail -40 gpurun_out/pytest_r04i.log; exit 1; }
tail -1 gpurun_out/pytest_r04i.log
for i in 1 2 3; do timeout -k 10 120 python tools/npg_phase.py time amp_extensions_amd/libamx_hip.so 40960 197 36 || exit 1; done > gpurun_out/r04i_npg_phase.txt 2>&1 || { tail -20 gpurun_out/r04i_npg_phase.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04i_npg_phase.txt
timeout -k 10 200 python tools/npg_time.py > gpurun_out/r04i_npg_time.txt 2>&1 || { tail -20 gpurun_out/r04i_npg_time.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04i_npg_time.txt | tail -3 | cut -c1-200

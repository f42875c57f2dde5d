#!/bin/bash
# r04f: the RFF pass with the register-resident epilogue (fast Cody-Waite cos = base; OCML cosf =
# cosf; round 3's LDS-staged epilogue = r3), interleaved, and the GPU tests that cover the RFF
# features (parity, h3, configs, share shapes, relabel).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_h3.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_share_shapes.py tests/test_gpu_relabel_fused.py tests/test_gpu_cost_inputs.py tests/test_gpu_npg.py > gpurun_out/pytest_r04f.log 2>&1 || { tail -40 gpurun_out/pytest_r04f.log; exit 1; }
tail -1 gpurun_out/pytest_r04f.log
for i in 1 2 3; do timeout -k 10 120 python tools/rff_ab.py base cosf r3 || exit 1; done > gpurun_out/r04f_rff_ab.txt 2>&1 || { tail -20 gpurun_out/r04f_rff_ab.txt; exit 1; }
RFF_ROWS=5120 timeout -k 10 120 python tools/rff_ab.py base cosf r3 >> gpurun_out/r04f_rff_ab.txt 2>&1 || { tail -20 gpurun_out/r04f_rff_ab.txt; exit 1; }
cat gpurun_out/r04f_rff_ab.txt | cut -c1-200

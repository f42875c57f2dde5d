#!/bin/bash
# r04h: the RFF pass on 128 x 256 16x16x32 split-schedule tiles (base) vs round 3's 128 x 128
# tiles (t0 = RFF_TILE 0) at 40 960 and 20 480 rows, and the RFF tile-shape parity tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_h3.py tests/test_gpu_configs.py tests/test_gpu_share_shapes.py > gpurun_out/pytest_r04h.log 2>&1 || { tail -40 gpurun_out/pytest_r04h.log; exit 1; }
tail -1 gpurun_out/pytest_r04h.log
for i in 1 2 3; do timeout -k 10 120 python tools/rff_ab.py base t0 || exit 1; done > gpurun_out/r04h_rff_ab.txt 2>&1 || { tail -20 gpurun_out/r04h_rff_ab.txt; exit 1; }
for i in 1 2; do RFF_ROWS=20480 timeout -k 10 120 python tools/rff_ab.py base t0 || exit 1; done >> gpurun_out/r04h_rff_ab.txt 2>&1 || { tail -20 gpurun_out/r04h_rff_ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04h_rff_ab.txt | cut -c1-200

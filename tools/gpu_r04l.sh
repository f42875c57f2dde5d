#!/bin/bash
# r04l: the 80 x 224 output tile with its A operand two K-tiles ahead (DEEPA, new) vs one (old)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; L=$R/amp_extensions_amd
cd "$R" && mkdir -p gpurun_out
cp $L/libamx_hip_new.so $L/libamx_hip.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_h3.py tests/test_gpu_share_shapes.py tests/test_gpu_out_ring.py > gpurun_out/pytest_r04l.log 2>&1 || { tail -40 gpurun_out/pytest_r04l.log; exit 1; }
tail -1 gpurun_out/pytest_r04l.log
bash tools/so_ab.sh 3 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --total-samples 5000 --expert-rows 6250 > gpurun_out/r04l_share5k_ab.txt 2>&1 || { tail -20 gpurun_out/r04l_share5k_ab.txt; exit 1; }
cp $L/libamx_hip_new.so $L/libamx_hip.so
for f in share5k; do echo "== $f"; grep -E '^==|"value"' gpurun_out/r04l_${f}_ab.txt | grep -v amdgpu | sed -E 's/.*"value": ([0-9.]+).*"ms_per_step": ([0-9.]+).*/\1 \2/'; done

#!/bin/bash
# r04y: the 160-row hidden tile (5120 lanes: the N = 4 / 8 shares) with its A operand two K-tiles
# ahead (new, HROW5_DEEPA 1) vs one (old): GEMM / share-shape / multirank tests, the N = 8 and N = 4
# share benches alternating old / new processes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; L=$R/amp_extensions_amd
cd "$R" && mkdir -p gpurun_out
cp $L/libamx_hip_new.so $L/libamx_hip.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_h3.py tests/test_gpu_share_shapes.py tests/test_gpu_multirank.py tests/test_gpu_out_ring.py > gpurun_out/pytest_r04y.log 2>&1 || { tail -40 gpurun_out/pytest_r04y.log; exit 1; }
tail -1 gpurun_out/pytest_r04y.log
bash tools/so_ab.sh 3 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --total-samples 5000 --expert-rows 6250 > gpurun_out/r04y_share5k_ab.txt 2>&1 || { tail -20 gpurun_out/r04y_share5k_ab.txt; exit 1; }
bash tools/so_ab.sh 2 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --total-samples 10000 --expert-rows 12500 > gpurun_out/r04y_share10k_ab.txt 2>&1 || { tail -20 gpurun_out/r04y_share10k_ab.txt; exit 1; }
cp $L/libamx_hip_new.so $L/libamx_hip.so
for f in share5k share10k; do echo "== $f"; grep -E '^==|"value"' gpurun_out/r04y_${f}_ab.txt | grep -v amdgpu | sed -E 's/.*"value": ([0-9.]+).*"ms_per_step": ([0-9.]+).*/\1 \2/'; done

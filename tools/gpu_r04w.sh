#!/bin/bash
# r04w: the RFF pass on 128 x 64 tiles at five workgroups per CU (new, RFF_OCC5 1: 2560 tiles in 2 rounds of 1280) vs 128 x 128 at three (old)
# RFF / MMD / parity tests, tools/rff_ab.py (40 960 and 21 504 rows), the default
# bench and the N = 8 share alternating old / new.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; L=$R/amp_extensions_amd
cd "$R" && mkdir -p gpurun_out
cp $L/libamx_hip_new.so $L/libamx_hip.so
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_h3.py tests/test_gpu_configs.py tests/test_gpu_share_shapes.py tests/test_gpu_relabel_fused.py tests/test_gpu_parity.py tests/test_gpu_cost_inputs.py tests/test_gpu_multirank.py tests/test_gpu_surfaces.py > gpurun_out/pytest_r04w.log 2>&1 || { tail -40 gpurun_out/pytest_r04w.log; exit 1; }
tail -1 gpurun_out/pytest_r04w.log
for i in 1 2 3; do timeout -k 10 120 python tools/rff_ab.py new old || exit 1; done > gpurun_out/r04w_rff_ab.txt 2>&1 || { tail -20 gpurun_out/r04w_rff_ab.txt; exit 1; }
RFF_ROWS=21504 timeout -k 10 120 python tools/rff_ab.py new old >> gpurun_out/r04w_rff_ab.txt 2>&1 || { tail -20 gpurun_out/r04w_rff_ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04w_rff_ab.txt | cut -c1-200
bash tools/so_ab.sh 3 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r04w_bench_ab.txt 2>&1 || { tail -20 gpurun_out/r04w_bench_ab.txt; exit 1; }
bash tools/so_ab.sh 2 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --total-samples 5000 --expert-rows 6250 > gpurun_out/r04w_share5k_ab.txt 2>&1 || { tail -20 gpurun_out/r04w_share5k_ab.txt; exit 1; }
cp $L/libamx_hip_new.so $L/libamx_hip.so
for f in bench share5k; do echo "== $f"; grep -E '^==|"value"' gpurun_out/r04w_${f}_ab.txt | grep -v amdgpu | sed -E 's/.*"value": ([0-9.]+).*"ms_per_step": ([0-9.]+).*/\1 \2/'; done

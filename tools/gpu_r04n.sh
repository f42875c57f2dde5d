#!/bin/bash
# r04n: the RFF pass as whole rounds of 128 x 128 tiles + one round of 128 x 64 tiles (new,
# RFF_SPLIT 1) vs one launch of 128 x 128 tiles (old): RFF tests, tools/rff_ab.py at 40 960 and
# 21 504 rows (the N = 1 and N = 2 shapes), and the default bench alternating old / new.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; L=$R/amp_extensions_amd
cd "$R" && mkdir -p gpurun_out
cp $L/libamx_hip_new.so $L/libamx_hip.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_h3.py tests/test_gpu_configs.py tests/test_gpu_share_shapes.py tests/test_gpu_relabel_fused.py tests/test_gpu_parity.py > gpurun_out/pytest_r04n.log 2>&1 || { tail -40 gpurun_out/pytest_r04n.log; exit 1; }
tail -1 gpurun_out/pytest_r04n.log
for i in 1 2 3; do timeout -k 10 120 python tools/rff_ab.py new old || exit 1; done > gpurun_out/r04n_rff_ab.txt 2>&1 || { tail -20 gpurun_out/r04n_rff_ab.txt; exit 1; }
for i in 1 2; do RFF_ROWS=21504 timeout -k 10 120 python tools/rff_ab.py new old || exit 1; done >> gpurun_out/r04n_rff_ab.txt 2>&1 || { tail -20 gpurun_out/r04n_rff_ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04n_rff_ab.txt | cut -c1-200
bash tools/so_ab.sh 3 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r04n_bench_ab.txt 2>&1 || { tail -20 gpurun_out/r04n_bench_ab.txt; exit 1; }
cp $L/libamx_hip_new.so $L/libamx_hip.so
grep -E '^==|"value"' gpurun_out/r04n_bench_ab.txt | grep -v amdgpu | sed -E 's/.*"value": ([0-9.]+).*"ms_per_step": ([0-9.]+).*/\1 \2/'

#!/bin/bash
# r04k: the 80 x 224 output tile at 5120 lanes (new) vs round 3's stream-K 128 x 224 (old): the
# GEMM tests at 5120 lanes, share shapes, multi-rank, sampler; then the N = 8 / N = 4 per-rank
# share benches alternating old / new processes (tools/so_ab.sh), and a rocprof timeline of new.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; L=$R/amp_extensions_amd
cd "$R" && mkdir -p gpurun_out
cp $L/libamx_hip_new.so $L/libamx_hip.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_h3.py tests/test_gpu_share_shapes.py tests/test_gpu_multirank.py tests/test_gpu_sampler.py tests/test_gpu_out_ring.py > gpurun_out/pytest_r04k.log 2>&1 || { tail -40 gpurun_out/pytest_r04k.log; exit 1; }
tail -1 gpurun_out/pytest_r04k.log
bash tools/so_ab.sh 3 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --total-samples 5000 --expert-rows 6250 > gpurun_out/r04k_share5k_ab.txt 2>&1 || { tail -20 gpurun_out/r04k_share5k_ab.txt; exit 1; }
bash tools/so_ab.sh 2 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --total-samples 10000 --expert-rows 12500 > gpurun_out/r04k_share10k_ab.txt 2>&1 || { tail -20 gpurun_out/r04k_share10k_ab.txt; exit 1; }
cp $L/libamx_hip_new.so $L/libamx_hip.so
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r04k_5k" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --total-samples 5000 --expert-rows 6250 --steps 10 --warmup 2 > "$R/gpurun_out/prof_r04k_5k.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_r04k_5k.log"; exit 1; }
cd "$R"
python tools/trace_timeline.py gpurun_out/prof_r04k_5k/run_kernel_trace.csv -2 1 > gpurun_out/r04k_timeline_5k.txt 2>&1
for f in share5k share10k; do echo "== $f"; grep -E '^==|"value"' gpurun_out/r04k_${f}_ab.txt | grep -v amdgpu | sed -E 's/.*"value": ([0-9.]+).*"ms_per_step": ([0-9.]+).*/\1 \2/'; done
cat gpurun_out/r04k_timeline_5k.txt

#!/bin/bash
# r04b: first run of the limb-format forward (amx_gemm_lb.hip): its tests, the f16x3 tests, then
# bench lines (default, N = 8 share) and a rocprofv3 kernel trace of the default bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lb.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_r04b_lb.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" gpurun_out/pytest_r04b_lb.log | head -40; tail -30 gpurun_out/pytest_r04b_lb.log; exit 1; }
tail -1 gpurun_out/pytest_r04b_lb.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_h3.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r04b_h3.log 2>&1; grep -E "^FAILED|passed|failed" gpurun_out/pytest_r04b_h3.log | head
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.err || { tail -20 gpurun_out/r04b_bench.err; exit 1; }
cut -c1-160 gpurun_out/r04b_bench.json; grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r04b_bench.json
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --total-samples 5000 --expert-rows 6250 > gpurun_out/r04b_share5k.json 2>&1 || { tail -20 gpurun_out/r04b_share5k.json; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r04b_share5k.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r04b" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 > "$R/gpurun_out/prof_r04b.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_r04b.log"; exit 1; }
cd "$R" && python tools/trace_summary.py gpurun_out/prof_r04b/run_kernel_trace.csv 125 | head -24

#!/bin/bash
set -o pipefail
TAG=${1:-pol}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_step_act.py tests/test_gpu_policy_shapes.py tests/test_gpu_gae.py tests/test_gpu_parity.py tests/test_gpu_h3.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest FAILED"; grep -E "FAILED|Error|assert" gpurun_out/pytest_$TAG.log | head -20; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
{ timeout -k 10 300 python -u tools/rollout_ab.py 8192 base,x1,a1 && timeout -k 10 300 python -u tools/rollout_ab.py 5120 base,x1,a1; } > gpurun_out/ab_$TAG.txt 2>&1 || { echo "ab FAILED"; tail -20 gpurun_out/ab_$TAG.txt; exit 1; }
cat gpurun_out/ab_$TAG.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv -- python "$R/tools/stepact_trace.py" 8192 > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_$TAG.log"; exit 1; }
grep -E "k_policy|k_assemble|k_step" "$R/gpurun_out/prof_$TAG/run_kernel_stats.csv" | cut -c1-200

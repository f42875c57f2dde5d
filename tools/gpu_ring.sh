#!/bin/bash
# Output-layer ring tile: its bit-identity / oracle tests, the forward A/B, and a short bench.
set -o pipefail
TAG=${1:-ring}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_out_ring.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest FAILED"; grep -E "FAILED|Error|assert" gpurun_out/pytest_$TAG.log | head -20; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python -u tools/out_ab.py 8192 5120 7168 > gpurun_out/out_ab_$TAG.txt 2>&1 || { echo "out_ab FAILED"; tail -20 gpurun_out/out_ab_$TAG.txt; exit 1; }
cat gpurun_out/out_ab_$TAG.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench FAILED"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-200
timeout -k 10 300 python bench.py --no-cpu-baseline --total-samples 5000 --expert-rows 6250 > gpurun_out/bench_${TAG}_5k.log 2>&1 || { echo "bench 5k FAILED"; tail -20 gpurun_out/bench_${TAG}_5k.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_5k.log | cut -c1-200

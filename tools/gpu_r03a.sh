#!/bin/bash
# Round-3 first pass: -m gpu suite, smoke, the default bench line, the reference-semantics
# (--mode paths) line, and the 2-rank launches (gloo and RCCL) on the one card.
set -o pipefail
TAG=${1:-r03a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest FAILED"; grep -E "FAILED|Error" gpurun_out/pytest_$TAG.log | head -20; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke FAILED"; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench FAILED"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-200
timeout -k 10 300 python bench.py --mode paths --no-cpu-baseline > gpurun_out/bench_${TAG}_paths.log 2>&1 || { echo "paths FAILED"; tail -20 gpurun_out/bench_${TAG}_paths.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_paths.log | cut -c1-200
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --no-cpu-baseline > gpurun_out/bench_${TAG}_g2gloo.log 2>&1 || { echo "g2 gloo FAILED"; tail -20 gpurun_out/bench_${TAG}_g2gloo.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_g2gloo.log | cut -c1-200

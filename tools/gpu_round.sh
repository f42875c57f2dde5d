#!/bin/bash
# One GPU-box pass: all -m gpu tests, smoke, the default bench line, and the bench at the
# strong-scaling per-rank shares (40000/N samples, N = 2, 4, 8).  Each GPU step runs under its
# own time limit; the chain stops at the first failure.  usage: tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest FAILED"; grep -E "FAILED|Error|error" gpurun_out/pytest_gpu_$TAG.log | head -20; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke FAILED"; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench FAILED"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-160
for n in 20000 10000 5000; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --total-samples $n > gpurun_out/bench_${TAG}_$n.log 2>&1 || { echo "bench $n FAILED"; tail -20 gpurun_out/bench_${TAG}_$n.log; exit 1; }
  tail -1 gpurun_out/bench_${TAG}_$n.log | cut -c1-160
done

#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, optionally rocprofv3 kernel stats (PROF=1).
# Every GPU step has its own time limit and the chain stops at the first failure.
# usage: tools/gpu_check.sh [tag] [extra bench args...]
set -o pipefail
TAG=${1:-run}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest FAILED"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke FAILED"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 500 python bench.py "$@" > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench FAILED"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
if [ "${PROF:-0}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 "$@" > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo "rocprof FAILED"; tail -20 "$R/gpurun_out/prof_$TAG.log"; exit 1; }
  echo "rocprof ok"
fi

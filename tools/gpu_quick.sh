#!/bin/bash
# Quick GPU pass: the given test files, the default bench line, the 5000-sample share, and a
# rocprofv3 kernel-stats run of the default bench (each step time-limited; stops at a failure).
# usage: tools/gpu_quick.sh TAG test_file...
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread "$@" > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest FAILED"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -1 gpurun_out/pytest_$TAG.log
fi
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench FAILED"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-140
timeout -k 10 200 python bench.py --no-cpu-baseline --total-samples 5000 > gpurun_out/bench_${TAG}_5000.log 2>&1 || { echo "bench 5000 FAILED"; tail -20 gpurun_out/bench_${TAG}_5000.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_5000.log | cut -c1-140
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo "rocprof FAILED"; tail -5 "$R/gpurun_out/prof_$TAG.log"; exit 1; }
echo "rocprof ok"

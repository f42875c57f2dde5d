#!/bin/bash
# Quick pass: optional test files, the strong-scaling share benches and a rocprofv3 trace of the
# 5000-sample share.  usage: tools/gpu_share.sh TAG [test files...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread "$@" > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest FAILED"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -1 gpurun_out/pytest_$TAG.log
fi
for n in 40000 20000 5000; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --total-samples $n > gpurun_out/bench_${TAG}_$n.log 2>&1 || { echo "bench $n FAILED"; tail -20 gpurun_out/bench_${TAG}_$n.log; exit 1; }
  tail -1 gpurun_out/bench_${TAG}_$n.log | cut -c1-120
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_5k" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --total-samples 5000 --steps 10 --warmup 2 > "$R/gpurun_out/prof_${TAG}_5k.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_${TAG}_5k.log"; exit 1; }
echo "prof ok"

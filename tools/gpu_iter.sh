#!/bin/bash
# Iteration pass: the whole -m gpu suite, the default bench line, the strong-scaling shares,
# and rocprofv3 kernel traces of the N = 1 and 5000-sample runs (each GPU step time-limited;
# the chain stops at the first failure).  usage: tools/gpu_iter.sh TAG
set -o pipefail
TAG=${1:-it}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest FAILED"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench FAILED"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-120
for n in 20000 10000 5000; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --total-samples $n > gpurun_out/bench_${TAG}_$n.log 2>&1 || { echo "bench $n FAILED"; tail -20 gpurun_out/bench_${TAG}_$n.log; exit 1; }
  tail -1 gpurun_out/bench_${TAG}_$n.log | cut -c1-120
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_8k" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 > "$R/gpurun_out/prof_${TAG}_8k.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_${TAG}_8k.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_5k" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --total-samples 5000 --steps 10 --warmup 2 > "$R/gpurun_out/prof_${TAG}_5k.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_${TAG}_5k.log"; exit 1; }
echo "prof ok"

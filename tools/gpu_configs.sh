#!/bin/bash
# Bench lines for the other BASELINE configs on the current build (1 GPU): configs[1] shape (4096
# lanes x 10 steps, MMD vs the 50 000-row expert buffer), the AMP pose-feature path (configs[4]'s
# per-GPU share), the LS-disc reward on [s, s'], and the scene layout S = 226 / A = 28.
set -o pipefail
TAG=${1:-cfg}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
run() {
  local name=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench_${TAG}_$name.log 2>&1 || { echo "bench $name FAILED"; tail -20 gpurun_out/bench_${TAG}_$name.log; exit 1; }
  tail -1 gpurun_out/bench_${TAG}_$name.log | cut -c1-120
}
run default
run c2 --lanes 4096
run amp --cost amp
run gail --cost gail
run c3faithful --faithful

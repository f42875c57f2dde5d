#!/bin/bash
# Round-end evidence pass (TAG, e.g. r02e): the -m gpu suite, smoke, the default bench line (with
# the CPU baseline), the strong-scaling share benches, rocprofv3 kernel traces of the N = 1 and
# 5000-sample runs, and the PMC HBM-traffic passes of the ensemble GEMM; each GPU step under its
# own time limit, the chain stops at the first failure.  Copy the results to profiles/ afterwards.
set -o pipefail
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest FAILED"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke FAILED"; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench FAILED"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-140
# per-rank shares of the strong-scaling runs (40000/N samples; with --expert-rows 50000/N the
# rank's sharded expert block, the serial all-reduce aside)
for spec in 20000:25000 10000:12500 5000:6250; do
  n=${spec%%:*}; e=${spec##*:}
  timeout -k 10 200 python bench.py --no-cpu-baseline --total-samples $n > gpurun_out/bench_${TAG}_$n.log 2>&1 || { echo "bench $n FAILED"; tail -20 gpurun_out/bench_${TAG}_$n.log; exit 1; }
  tail -1 gpurun_out/bench_${TAG}_$n.log | cut -c1-140
  timeout -k 10 200 python bench.py --no-cpu-baseline --total-samples $n --expert-rows $e > gpurun_out/bench_${TAG}_${n}_e$e.log 2>&1 || { echo "bench $n/$e FAILED"; tail -20 gpurun_out/bench_${TAG}_${n}_e$e.log; exit 1; }
  tail -1 gpurun_out/bench_${TAG}_${n}_e$e.log | cut -c1-140
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_8k" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 > "$R/gpurun_out/prof_${TAG}_8k.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_${TAG}_8k.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_5k" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --total-samples 5000 --steps 10 --warmup 2 > "$R/gpurun_out/prof_${TAG}_5k.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_${TAG}_5k.log"; exit 1; }
cd "$R" && bash tools/pmc_traffic.sh $TAG f16x3

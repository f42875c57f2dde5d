#!/bin/bash
# Round-3 evidence pass (TAG): the -m gpu suite, smoke, the bench line as the driver runs it
# (--gpus 1 --steps 20 --warmup 5, with the CPU baseline), the reference-semantics line, the
# strong-scaling per-rank shares, the other BASELINE configs, rocprofv3 kernel traces of the
# N = 1 and N = 8-share runs, and the PMC HBM-traffic passes.  Each GPU step under its own time
# limit; the chain stops at the first failure.  Copy the results to profiles/ afterwards.
set -o pipefail
TAG=${1:-r03b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest FAILED"; grep -E "FAILED|Error" gpurun_out/pytest_$TAG.log | head -20; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke FAILED"; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench FAILED"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-160
timeout -k 10 300 python bench.py --mode paths --no-cpu-baseline > gpurun_out/bench_${TAG}_paths.log 2>&1 || { echo "paths FAILED"; tail -20 gpurun_out/bench_${TAG}_paths.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_paths.log | cut -c1-160
for spec in 20000:25000 10000:12500 5000:6250; do
  n=${spec%%:*}; e=${spec##*:}
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --total-samples $n --expert-rows $e > gpurun_out/bench_${TAG}_share_${n}_e$e.log 2>&1 || { echo "bench $n FAILED"; tail -20 gpurun_out/bench_${TAG}_share_${n}_e$e.log; exit 1; }
  tail -1 gpurun_out/bench_${TAG}_share_${n}_e$e.log | cut -c1-140
done
bash tools/gpu_configs.sh ${TAG}_cfg || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_8k" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 > "$R/gpurun_out/prof_${TAG}_8k.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_${TAG}_8k.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_5k" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --total-samples 5000 --expert-rows 6250 --steps 10 --warmup 2 > "$R/gpurun_out/prof_${TAG}_5k.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_${TAG}_5k.log"; exit 1; }
cd "$R" && bash tools/pmc_traffic.sh $TAG f16x3

#!/bin/bash
# r03e (2): the -m gpu suite + smoke on the build with the 8-deep feature-message / partial-sum
# loads, then rocprofv3 kernel stats of the default bench, old build vs new, and the bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; L=$R/amp_extensions_amd
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r03e.log 2>&1 || { tail -30 gpurun_out/pytest_r03e.log; exit 1; }
tail -1 gpurun_out/pytest_r03e.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r03e.log 2>&1 || { tail -20 gpurun_out/smoke_r03e.log; exit 1; }
tail -1 gpurun_out/smoke_r03e.log
cd /tmp && export TMPDIR=/tmp
for v in old new; do
  cp $L/libamx_hip_$v.so $L/libamx_hip.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r03e_$v" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 > "$R/gpurun_out/prof_r03e_$v.log" 2>&1 || { echo "rocprof $v failed"; tail -5 "$R/gpurun_out/prof_r03e_$v.log"; exit 1; }
done
cd "$R"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03e_bench.json 2> gpurun_out/r03e_bench.err || { tail -20 gpurun_out/r03e_bench.err; exit 1; }
cut -c1-200 gpurun_out/r03e_bench.json
for v in old new; do echo "== $v"; f=$(find gpurun_out/prof_r03e_$v -name "*kernel_stats.csv" | head -1); grep -E "feature_message|sum_partials|k_step|mmd_relabel" "$f" | cut -c1-200; done

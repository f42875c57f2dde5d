#!/bin/bash
# rocprofv3 kernel traces of bench.py at the per-rank shares of the strong-scaling runs
# (40000 / N samples per rank, N = 1, 2, 4, 8), each step under its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
for n in 5000 10000 20000; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --total-samples $n --steps 20 --warmup 3 > gpurun_out/bench_share_$n.log 2>&1 || { echo "bench $n failed"; tail -5 gpurun_out/bench_share_$n.log; exit 1; }
  tail -1 gpurun_out/bench_share_$n.log | cut -c1-200
done
cd /tmp && export TMPDIR=/tmp
for n in 5000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_share_$n" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --total-samples $n --steps 10 --warmup 2 > "$R/gpurun_out/prof_share_$n.log" 2>&1 || { echo "rocprof $n failed"; tail -5 "$R/gpurun_out/prof_share_$n.log"; exit 1; }
done
echo done

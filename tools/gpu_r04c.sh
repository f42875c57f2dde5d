#!/bin/bash
# r04c: register-staged limb forward: tests, then bench A/B: limbs (registers) / limbs (DMA) / f32
# format (h3), default and N = 8 share, alternating processes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lb.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r04c_lb.log 2>&1 || { tail -30 gpurun_out/pytest_r04c_lb.log; exit 1; }
tail -1 gpurun_out/pytest_r04c_lb.log
for i in 1; do
  for v in "--act-format limbs" "--act-format limbs --lb-stage 1" "--act-format f32"; do
    for n in 40000 5000; do
      timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --total-samples $n --expert-rows $((n * 50000 / 40000)) $v > gpurun_out/r04c_b.json 2>&1 || { tail -20 gpurun_out/r04c_b.json; exit 1; }
      echo "$v n=$n $(grep -o '"value": [0-9.]*' gpurun_out/r04c_b.json) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r04c_b.json)"
    done
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r04c" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 > "$R/gpurun_out/prof_r04c.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_r04c.log"; exit 1; }
cd "$R" && python tools/trace_summary.py gpurun_out/prof_r04c/run_kernel_trace.csv 125 | head -12

#!/bin/bash
# r04r: the NPG update's host glue folded into kernels (curvature, whitening, step + clamp):
# NPG / GAE GPU tests, the update time, its kernel timeline, and the --mode train bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_npg.py tests/test_gpu_gae.py > gpurun_out/pytest_r04r.log 2>&1 || { tail -40 gpurun_out/pytest_r04r.log; exit 1; }
tail -1 gpurun_out/pytest_r04r.log
timeout -k 10 200 python tools/npg_time.py > gpurun_out/r04r_npg_time.txt 2>&1 || { tail -20 gpurun_out/r04r_npg_time.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04r_npg_time.txt | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r04r" -o run --output-format csv -- python "$R/tools/npg_time.py" > "$R/gpurun_out/prof_r04r.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_r04r.log"; exit 1; }
cd "$R"
timeout -k 10 400 python bench.py --mode train --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r04r_bench_train.json 2> gpurun_out/r04r_bench_train.err || { tail -20 gpurun_out/r04r_bench_train.err; exit 1; }
cut -c1-300 gpurun_out/r04r_bench_train.json

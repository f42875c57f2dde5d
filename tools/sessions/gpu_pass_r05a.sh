set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_motion.py tests/test_gpu_sampler.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05a_pytest.log 2>&1 || { tail -40 gpurun_out/r05a_pytest.log; exit 1; }
tail -1 gpurun_out/r05a_pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r05a_bench.json 2> gpurun_out/r05a_bench.err || { tail -20 gpurun_out/r05a_bench.err; exit 1; }
cut -c1-200 gpurun_out/r05a_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r05a" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --steps 20 --warmup 5 > "$R/gpurun_out/prof_r05a.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_r05a.log"; exit 1; }
cd "$R"
python tools/trace_summary.py gpurun_out/prof_r05a/run_kernel_trace.csv 500 > gpurun_out/r05a_trace_summary.txt 2>&1
head -4 gpurun_out/r05a_trace_summary.txt
grep -o '"avg_launch_us": [0-9.]*' gpurun_out/prof_r05a.log gpurun_out/r05a_bench.json

set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_npg.py tests/test_gpu_gae.py > gpurun_out/r05c_pytest.log 2>&1 || { tail -40 gpurun_out/r05c_pytest.log; exit 1; }
tail -1 gpurun_out/r05c_pytest.log
timeout -k 10 200 python tools/npg_time.py > gpurun_out/r05c_npg_time.txt 2>&1 || { tail -20 gpurun_out/r05c_npg_time.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r05c_npg_time.txt | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r05c" -o run --output-format csv -- python "$R/tools/npg_time.py" > "$R/gpurun_out/prof_r05c.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_r05c.log"; exit 1; }
cd "$R"
python tools/npg_timeline.py gpurun_out/prof_r05c/run_kernel_trace.csv > gpurun_out/r05c_npg_timeline.txt
tail -14 gpurun_out/r05c_npg_timeline.txt
timeout -k 10 400 python bench.py --mode train --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r05c_bench_train.json 2> gpurun_out/r05c_bench_train.err || { tail -20 gpurun_out/r05c_bench_train.err; exit 1; }
cut -c1-200 gpurun_out/r05c_bench_train.json

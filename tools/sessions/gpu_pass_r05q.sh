# r05q: advantage whitening over the chip (two launches): GAE / NPG tests, NPG update time, its kernel timeline,
# the training-mode bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gae.py tests/test_gpu_npg.py > gpurun_out/r05q_pytest.log 2>&1 || { tail -40 gpurun_out/r05q_pytest.log; exit 1; }
tail -1 gpurun_out/r05q_pytest.log
timeout -k 10 300 python tools/npg_time.py > gpurun_out/r05q_npg_time.txt 2>&1 || { tail -5 gpurun_out/r05q_npg_time.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r05q_npg_time.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r05q" -o run --output-format csv -- python "$R/tools/npg_time.py" > "$R/gpurun_out/prof_r05q.log" 2>&1 || { echo "rocprof failed"; exit 1; }
cd "$R" && python tools/npg_timeline.py gpurun_out/prof_r05q/run_kernel_trace.csv > gpurun_out/r05q_npg_timeline.txt && grep -E "whiten|update span" gpurun_out/r05q_npg_timeline.txt | head -5
timeout -k 10 300 python bench.py --mode train --no-cpu-baseline > gpurun_out/r05q_bench_train.json 2>/dev/null || { echo "train bench failed"; exit 1; }
cut -c1-160 gpurun_out/r05q_bench_train.json

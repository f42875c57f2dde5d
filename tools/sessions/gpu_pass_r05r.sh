# r05r: NPG update glue (curvature folded into the CG start; no concatenation kernel in the read-back):
# GAE / NPG tests, update time, timeline, training-mode bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gae.py tests/test_gpu_npg.py > gpurun_out/r05r_pytest.log 2>&1 || { tail -40 gpurun_out/r05r_pytest.log; exit 1; }
tail -1 gpurun_out/r05r_pytest.log
timeout -k 10 300 python tools/npg_time.py > gpurun_out/r05r_npg_time.txt 2>&1 || { tail -5 gpurun_out/r05r_npg_time.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r05r_npg_time.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r05r" -o run --output-format csv -- python "$R/tools/npg_time.py" > "$R/gpurun_out/prof_r05r.log" 2>&1 || { echo "rocprof failed"; exit 1; }
cd "$R" && python tools/npg_timeline.py gpurun_out/prof_r05r/run_kernel_trace.csv > gpurun_out/r05r_npg_timeline.txt && grep -E "update span" gpurun_out/r05r_npg_timeline.txt
for i in 1 2; do
timeout -k 10 300 python bench.py --mode train --no-cpu-baseline > gpurun_out/r05r_bench_train_$i.json 2>/dev/null || { echo "train bench failed"; exit 1; }
cut -c1-140 gpurun_out/r05r_bench_train_$i.json
done

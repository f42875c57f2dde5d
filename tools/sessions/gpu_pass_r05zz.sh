# r05zz: final evidence pass of round 5 after the late changes (feature message, relabel block order, eager shares): every GPU test (shipped library), smoke(), the experimental A/B tests on an
# AMX_EXPERIMENTAL=1 build (libamx_hip_exp.so, swapped in and restored), the default bench line, its timed-region
# rocprof summary, the N = 4 / 8 share lines and the training-mode line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05zz_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r05zz_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r05zz_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05zz_smoke.log 2>&1 || { tail -20 gpurun_out/r05zz_smoke.log; exit 1; }
tail -2 gpurun_out/r05zz_smoke.log
cp amp_extensions_amd/libamx_hip.so /tmp/libamx_orig.so && cp amp_extensions_amd/libamx_hip_exp.so amp_extensions_amd/libamx_hip.so
timeout -k 10 600 python -u -m pytest tests -m "gpu and experimental" -x -q --timeout 300 --timeout-method thread > gpurun_out/r05zz_pytest_experimental.log 2>&1; rc=$?
cp /tmp/libamx_orig.so amp_extensions_amd/libamx_hip.so
tail -2 gpurun_out/r05zz_pytest_experimental.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r05zz_bench.json 2> gpurun_out/r05zz_bench.err || { tail -20 gpurun_out/r05zz_bench.err; exit 1; }
cut -c1-300 gpurun_out/r05zz_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r05zz" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --steps 20 --warmup 5 > "$R/gpurun_out/prof_r05zz.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_r05zz.log"; exit 1; }
cd "$R"
python tools/trace_summary.py gpurun_out/prof_r05zz/run_kernel_trace.csv 500 > gpurun_out/r05zz_trace_summary.txt 2>&1
head -4 gpurun_out/r05zz_trace_summary.txt
grep -o '"avg_launch_us": [0-9.]*\|"frac": [0-9.]*' gpurun_out/prof_r05zz.log | head -4
for n in 5000 10000; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --total-samples $n --expert-rows $((50000 * n / 40000)) --steps 50 --warmup 10 > gpurun_out/r05zz_share_$n.json 2>/dev/null || { echo "share $n failed"; exit 1; }
  echo "share $n: $(cut -c1-120 gpurun_out/r05zz_share_$n.json)"
done
timeout -k 10 300 python bench.py --mode train --no-cpu-baseline > gpurun_out/r05zz_bench_train.json 2>/dev/null || { echo "train bench failed"; exit 1; }
cut -c1-140 gpurun_out/r05zz_bench_train.json

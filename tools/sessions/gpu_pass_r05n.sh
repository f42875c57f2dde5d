# r05n: evidence on the tree with the GEMM sources final for the round: every GPU test, smoke(), the HBM-traffic
# PMC record of the shipped GEMM build, the default bench line, its timed-region rocprof summary, share lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05n_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r05n_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r05n_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05n_smoke.log 2>&1 || { tail -20 gpurun_out/r05n_smoke.log; exit 1; }
tail -2 gpurun_out/r05n_smoke.log
timeout -k 10 700 bash tools/pmc_traffic.sh r05n f16x3 > gpurun_out/r05n_pmc_traffic.log 2>&1 || { tail -20 gpurun_out/r05n_pmc_traffic.log; exit 1; }
tail -1 gpurun_out/r05n_pmc_traffic.log
cp gpurun_out/gemm_traffic_f16x3.json amp_extensions_amd/data/gemm_traffic_f16x3.json
timeout -k 10 400 python bench.py > gpurun_out/r05n_bench.json 2> gpurun_out/r05n_bench.err || { tail -20 gpurun_out/r05n_bench.err; exit 1; }
cut -c1-300 gpurun_out/r05n_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r05n" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --steps 20 --warmup 5 > "$R/gpurun_out/prof_r05n.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_r05n.log"; exit 1; }
cd "$R"
python tools/trace_summary.py gpurun_out/prof_r05n/run_kernel_trace.csv 500 > gpurun_out/r05n_trace_summary.txt 2>&1
head -4 gpurun_out/r05n_trace_summary.txt
grep -o '"avg_launch_us": [0-9.]*\|"frac": [0-9.]*' gpurun_out/prof_r05n.log | head -4
for n in 5000 10000; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --total-samples $n --expert-rows $((50000 * n / 40000)) --steps 50 --warmup 10 > gpurun_out/r05n_share_$n.json 2>/dev/null || { echo "share $n failed"; exit 1; }
  echo "share $n: $(cut -c1-120 gpurun_out/r05n_share_$n.json)"
done

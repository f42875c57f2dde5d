#!/bin/bash
# r04z: the round-4 evidence pass on the final tree (re-run after each GEMM-source change: the traffic record is keyed to them) -- the whole -m gpu suite and smoke; the PMC
# HBM-traffic passes of the ensemble GEMM (their JSON goes to amp_extensions_amd/data/, where
# bench.py reads it, keyed to the GEMM sources' hash); the timed-region rocprofv3 kernel trace of
# the default bench; SQ counters of a hidden and the output layer; the default bench line (CPU
# baseline included); the N = 8 / 4 per-rank share lines; the NPG update time.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; L=$R/amp_extensions_amd
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r04z.log 2>&1; rc=$?
[ $rc -le 1 ] || { tail -40 gpurun_out/pytest_r04z.log; exit 1; }
grep -E "^FAILED|^ERROR" gpurun_out/pytest_r04z.log; tail -1 gpurun_out/pytest_r04z.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04z.log 2>&1 || { tail -20 gpurun_out/smoke_r04z.log; exit 1; }
tail -1 gpurun_out/smoke_r04z.log
bash tools/pmc_traffic.sh r04z f16x3 > gpurun_out/r04z_pmc.txt 2>&1 || { tail -20 gpurun_out/r04z_pmc.txt; exit 1; }
tail -1 gpurun_out/r04z_pmc.txt
cp gpurun_out/gemm_traffic_f16x3.json $L/data/gemm_traffic_f16x3.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r04z" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 > "$R/gpurun_out/prof_r04z.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_r04z.log"; exit 1; }
cd "$R"
python tools/trace_summary.py gpurun_out/prof_r04z/run_kernel_trace.csv 125 > gpurun_out/r04z_trace_summary.txt 2>&1 || { tail -5 gpurun_out/r04z_trace_summary.txt; exit 1; }
head -4 gpurun_out/r04z_trace_summary.txt
bash tools/h3_pmc.sh 3 > gpurun_out/r04z_sq_hidden3.txt 2>&1 || { tail -10 gpurun_out/r04z_sq_hidden3.txt; exit 1; }
bash tools/h3_pmc.sh 4 > gpurun_out/r04z_sq_output.txt 2>&1 || { tail -10 gpurun_out/r04z_sq_output.txt; exit 1; }
timeout -k 10 500 python bench.py > gpurun_out/r04z_bench.json 2> gpurun_out/r04z_bench.err || { tail -20 gpurun_out/r04z_bench.err; exit 1; }
cut -c1-400 gpurun_out/r04z_bench.json
timeout -k 10 200 python bench.py --no-cpu-baseline --total-samples 5000 --expert-rows 6250 > gpurun_out/r04z_share_n8.json 2>/dev/null || { echo "share n8 failed"; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --total-samples 10000 --expert-rows 12500 > gpurun_out/r04z_share_n4.json 2>/dev/null || { echo "share n4 failed"; exit 1; }
timeout -k 10 200 python tools/npg_time.py > gpurun_out/r04z_npg_time.txt 2>&1 || { tail -20 gpurun_out/r04z_npg_time.txt; exit 1; }
tail -3 gpurun_out/r04z_npg_time.txt | cut -c1-200

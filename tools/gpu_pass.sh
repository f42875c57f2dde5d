#!/bin/bash
# One parameterised GPU pass (replaces round 5's per-pass one-off scripts).  Run on the GPU box
# from the repository root:
#
#   bash tools/gpu_pass.sh TAG STEP [STEP ...]
#
# Every output goes to gpurun_out/TAG_*; copy what is judged into profiles/.  Steps (in the
# order given; the pass stops at the first failure, every GPU step under its own time limit):
#   tests[:EXPR]   pytest -m gpu (EXPR: a -k expression; tests:FILE.py runs one file)
#   smoke          __graft_entry__.smoke()
#   bench          the default bench line (driver configuration: 20 steps, 5 warmup)
#   prof           rocprofv3 --kernel-trace --stats of bench (no CPU leg) + the timed-region summary
#   shares         the N = 8 / 4 per-rank share lines (5000 / 10000 samples)
#   train          bench --mode train
#   paths          bench --mode paths (the drop-in sample_points + relabel_paths)
#   pathsprof      rocprofv3 --kernel-trace --stats of bench --mode paths (per-kernel totals vs the wall)
#   configs        the other BASELINE configs (tools/gpu_configs.sh)
#   timeline       per-launch timeline of the N = 8 share (tools/trace_timeline.py)
#   py:SCRIPT[:ARGS]  python tools/SCRIPT ARGS (comma-separated; an A/B or timing tool), output to TAG_SCRIPT.txt
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
O="gpurun_out/${TAG}"
for step in "$@"; do
  case "$step" in
    tests|tests:*)
      sel=${step#tests}; sel=${sel#:}
      if [[ "$sel" == *.py ]]; then args=("tests/$sel"); elif [ -n "$sel" ]; then args=(tests -k "$sel"); else args=(tests); fi
      timeout -k 10 1100 python -u -m pytest "${args[@]}" -m gpu -x -q --timeout 300 --timeout-method thread \
        > "${O}_pytest_gpu.log" 2>&1 || { tail -40 "${O}_pytest_gpu.log"; exit 1; }
      tail -2 "${O}_pytest_gpu.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "${O}_smoke.log" 2>&1 \
        || { tail -20 "${O}_smoke.log"; exit 1; }
      tail -2 "${O}_smoke.log" ;;
    bench)
      timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "${O}_bench.json" 2> "${O}_bench.err" \
        || { tail -20 "${O}_bench.err"; exit 1; }
      cut -c1-300 "${O}_bench.json" ;;
    prof)
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/${O}_prof" -o run \
          --output-format csv -- python "$R/bench.py" --no-cpu-baseline --steps 20 --warmup 5 > "$R/${O}_prof.log" 2>&1 ) \
        || { echo "rocprof failed"; tail -5 "${O}_prof.log"; exit 1; }
      python tools/trace_summary.py "${O}_prof/run_kernel_trace.csv" 500 > "${O}_trace_summary.txt" 2>&1
      cp "${O}_prof/run_kernel_stats.csv" "${O}_kernel_stats.csv" 2>/dev/null
      head -4 "${O}_trace_summary.txt"
      grep -o '"avg_launch_us": [0-9.]*\|"frac": [0-9.]*' "${O}_prof.log" | head -4 ;;
    shares)
      for n in 5000 10000; do
        timeout -k 10 200 python bench.py --no-cpu-baseline --total-samples $n --expert-rows $((50000 * n / 40000)) \
          --steps 50 --warmup 10 > "${O}_share_$n.json" 2>"${O}_share_$n.err" || { echo "share $n failed"; tail -5 "${O}_share_$n.err"; exit 1; }
        echo "share $n: $(cut -c1-160 "${O}_share_$n.json")"
      done ;;
    train)
      timeout -k 10 300 python bench.py --mode train --no-cpu-baseline > "${O}_bench_train.json" 2>"${O}_train.err" \
        || { echo "train bench failed"; tail -5 "${O}_train.err"; exit 1; }
      cut -c1-160 "${O}_bench_train.json" ;;
    paths)
      timeout -k 10 300 python bench.py --mode paths --no-cpu-baseline > "${O}_bench_paths.json" 2>"${O}_paths.err" \
        || { echo "paths bench failed"; tail -5 "${O}_paths.err"; exit 1; }
      cut -c1-200 "${O}_bench_paths.json" ;;
    pathsprof)
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/${O}_pprof" -o run \
          --output-format csv -- python "$R/bench.py" --mode paths --no-cpu-baseline > "$R/${O}_pprof.log" 2>&1 ) \
        || { echo "rocprof (paths) failed"; tail -5 "${O}_pprof.log"; exit 1; }
      cp "${O}_pprof/run_kernel_stats.csv" "${O}_paths_kernel_stats.csv" 2>/dev/null
      python tools/trace_summary.py "${O}_pprof/run_kernel_trace.csv" > "${O}_paths_trace_summary.txt" 2>&1
      head -24 "${O}_paths_trace_summary.txt" ;;
    configs)
      timeout -k 10 900 bash tools/gpu_configs.sh "${TAG}" > "${O}_configs.log" 2>&1 || { tail -20 "${O}_configs.log"; exit 1; }
      tail -8 "${O}_configs.log" ;;
    timeline)
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/${O}_tl" -o run \
          --output-format csv -- python "$R/bench.py" --no-cpu-baseline --total-samples 5000 --expert-rows 6250 \
          --steps 20 --warmup 5 > "$R/${O}_tl.log" 2>&1 ) || { echo "timeline trace failed"; exit 1; }
      python tools/trace_timeline.py "${O}_tl/run_kernel_trace.csv" > "${O}_timeline_share.txt" 2>&1
      head -20 "${O}_timeline_share.txt" ;;
    py:*)
      spec=${step#py:}; script=${spec%%:*}; rest=""; [[ "$spec" == *:* ]] && rest=${spec#*:}; rest=${rest//,/ }
      timeout -k 10 600 python -u "tools/$script" $rest > "${O}_${script%.py}.txt" 2>&1 \
        || { tail -20 "${O}_${script%.py}.txt"; exit 1; }
      tail -15 "${O}_${script%.py}.txt" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done

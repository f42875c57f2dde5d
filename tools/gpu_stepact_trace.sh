#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_stepact" -o run --output-format csv -- python "$R/tools/stepact_trace.py" 8192 > "$R/gpurun_out/prof_stepact.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_stepact.log"; exit 1; }
echo done

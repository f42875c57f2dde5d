#!/bin/bash
# r04q: kernel trace of the device NPG update (tools/npg_time.py under rocprofv3 --kernel-trace)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r04q" -o run --output-format csv -- python "$R/tools/npg_time.py" > "$R/gpurun_out/prof_r04q.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_r04q.log"; exit 1; }
cd "$R"
tail -2 gpurun_out/prof_r04q.log | cut -c1-200

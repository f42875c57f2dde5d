#!/bin/bash
# NPG pass kernel: kernel-trace profile of tools/npg_time.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_npg2 -o run -- python3 $R/tools/npg_time.py 40960 197 36 4 > $O/prof_npg2.log 2>&1 || { tail -20 $O/prof_npg2.log; exit 1; }
find $O/prof_npg2 -name '*stats*'
f=$(find $O/prof_npg2 -name '*kernel_stats.csv' | head -1)
head -8 "$f"

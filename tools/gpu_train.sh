#!/bin/bash
# bench.py --mode train (rollout + relabel + GAE + NPG update per step) and its kernel profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
T=${1:-train}
mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --mode train --steps 20 --warmup 3 > $O/${T}_bench.log 2>&1 || { tail -20 $O/${T}_bench.log; exit 1; }
tail -1 $O/${T}_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${T} -o run --output-format csv -- python3 $R/bench.py --mode train --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_${T}.log 2>&1 || { tail -20 $O/prof_${T}.log; exit 1; }
f=$(find $O/prof_${T} -name 'run_kernel_stats.csv' | head -1)
head -16 "$f" | cut -c1-150

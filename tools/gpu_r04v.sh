#!/bin/bash
# r04v: --mode paths (reference-semantics sample_points + relabel_paths) on the round-3 tree (_r3tree,
# a git worktree of 5cdcd73) vs the current tree, alternating processes on one box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
for i in 1 2; do
  for t in r3 now; do
    d=$R; [ $t = r3 ] && d=$R/_r3tree
    (cd $d && timeout -k 10 300 python bench.py --mode paths --no-cpu-baseline 2>/dev/null | tail -1 | sed -E "s/.*\"value\": ([0-9.]+).*/$t \1/") || exit 1
  done
done

#!/bin/bash
# The N = 8 per-rank share (5000 samples, 6250 expert rows) and the N = 1 default bench in one
# line each: value and ms per rollout (an A/B body for tools/so_ab.sh or tools/flag_ab.sh).
#   bash tools/bench_pair.sh [extra bench.py args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
s=$(timeout -k 10 200 python bench.py --no-cpu-baseline --total-samples 5000 --expert-rows 6250 --steps 50 --warmup 10 "$@" 2>/dev/null) || exit 1
n=$(timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 "$@" 2>/dev/null) || exit 1
v() { python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_us'))" "$1"; }
echo "share $(v "$s") | n1 $(v "$n")"

#!/bin/bash
# Alternate bench.py flag sets process by process on one box: tools/flag_ab.sh ROUNDS "ARGS A" "ARGS B" ...
# (each ARGS string is appended to `python bench.py --no-cpu-baseline`); prints value / GEMM average per run.
set -o pipefail
N=$1; shift
for i in $(seq $N); do
  for args in "$@"; do
    out=$(timeout -k 10 300 python bench.py --no-cpu-baseline $args 2>/dev/null) || { echo "FAILED: $args"; exit 1; }
    echo "== [$args] $(echo "$out" | grep -o '"value": [0-9.e+]*\|"avg_launch_us": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"
  done
done

#!/bin/bash
# Same-box A/B of library builds on bench.py lines: for each round and tag, install
# libamx_hip_<tag>.so and run bench.py with the given arguments; prints tag, value, ms_per_step and
# the GEMM timer's avg launch.  usage: tools/ab_bench.sh "<tags>" <rounds> <bench args...>
set -o pipefail
tags=$1; rounds=$2; shift 2
cp amp_extensions_amd/libamx_hip.so /tmp/libamx_hip_orig.so
for r in $(seq 1 $rounds); do
  for t in $tags; do
    cp amp_extensions_amd/libamx_hip_$t.so amp_extensions_amd/libamx_hip.so
    out=$(timeout -k 10 200 python bench.py --no-cpu-baseline "$@" 2>/dev/null | tail -1) || { echo "$t FAILED"; cp /tmp/libamx_hip_orig.so amp_extensions_amd/libamx_hip.so; exit 1; }
    echo "$t r$r $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_us"])')"
  done
done
cp /tmp/libamx_hip_orig.so amp_extensions_amd/libamx_hip.so

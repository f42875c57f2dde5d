#!/bin/bash
# r04s: the whole -m gpu suite, smoke and the default bench line on the final tree
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r04s.log 2>&1; rc=$?
[ $rc -le 1 ] || { tail -40 gpurun_out/pytest_r04s.log; exit 1; }
grep -E "^FAILED|^ERROR" gpurun_out/pytest_r04s.log; tail -1 gpurun_out/pytest_r04s.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04s.log 2>&1 || { tail -20 gpurun_out/smoke_r04s.log; exit 1; }
tail -1 gpurun_out/smoke_r04s.log
timeout -k 10 500 python bench.py > gpurun_out/r04s_bench.json 2> gpurun_out/r04s_bench.err || { tail -20 gpurun_out/r04s_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r04s_bench.json')); c=d['cpu_baseline']; r=d['roofline']; print(d['value'], r['frac'], r['traffic'], c['value'], c['spread'])"

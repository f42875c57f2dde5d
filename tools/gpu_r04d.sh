#!/bin/bash
# r04d: the whole -m gpu suite (reset noise, limb option, sampler fixes), smoke
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r04d.log 2>&1; rc=$?
[ $rc -le 1 ] || { tail -40 gpurun_out/pytest_r04d.log; exit 1; }
grep -E "^FAILED|^ERROR" gpurun_out/pytest_r04d.log; tail -1 gpurun_out/pytest_r04d.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04d.log 2>&1 || { tail -20 gpurun_out/smoke_r04d.log; exit 1; }
tail -1 gpurun_out/smoke_r04d.log

#!/bin/bash
# Fused step + next action: its bit-identity / oracle tests, the policy and rollout suites, the bench A/B.
set -o pipefail
TAG=${1:-stepact}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_step_act.py tests/test_gpu_policy_shapes.py tests/test_gpu_h3.py tests/test_gpu_share_shapes.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest FAILED"; grep -E "FAILED|Error|assert" gpurun_out/pytest_$TAG.log | head -20; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
{ timeout -k 10 300 python -u tools/rollout_ab.py 8192 base,a0,w8 && timeout -k 10 300 python -u tools/rollout_ab.py 5120 base,a0,w8; } > gpurun_out/stepact_ab_$TAG.txt 2>&1 || { echo "ab FAILED"; tail -20 gpurun_out/stepact_ab_$TAG.txt; exit 1; }
cat gpurun_out/stepact_ab_$TAG.txt

#!/bin/bash
# 2-rank rehearsal on one card: the multirank GPU test, then bench.py as 2 gloo ranks sharing the
# GPU at the 10000-sample total (5120 x 1 per rank: graph replay), overlapped and not.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multirank.py > gpurun_out/pytest_dist2.log 2>&1 || { echo "pytest FAILED"; tail -40 gpurun_out/pytest_dist2.log; exit 1; }
tail -1 gpurun_out/pytest_dist2.log
for ov in on off; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --total-samples 10000 --no-cpu-baseline --steps 10 --warmup 2 --overlap $ov > gpurun_out/bench_dist2_$ov.log 2>&1 || { echo "bench $ov FAILED"; tail -30 gpurun_out/bench_dist2_$ov.log; exit 1; }
  grep '"metric"' gpurun_out/bench_dist2_$ov.log | cut -c1-200
done

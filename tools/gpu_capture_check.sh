#!/bin/bash
# Graph-capture checks on one GPU: the graph-replay tests, the one-rank RCCL rehearsal under
# torchrun and a torchrun bench of the 8-GPU per-rank share (each step time-limited).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_h3.py -k "graph or multirank or rank" > gpurun_out/pt_cap.log 2>&1 || { echo "pytest FAILED"; tail -30 gpurun_out/pt_cap.log; exit 1; }
tail -1 gpurun_out/pt_cap.log
timeout -k 10 200 python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 tools/rccl_rehearsal.py > gpurun_out/rccl_cap.log 2>&1 || { echo "rehearsal FAILED"; tail -30 gpurun_out/rccl_cap.log; exit 1; }
grep "rccl rehearsal" gpurun_out/rccl_cap.log
timeout -k 10 200 python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --total-samples 5000 --steps 10 --warmup 3 > gpurun_out/bench_tr1.log 2>&1 || { echo "bench FAILED"; tail -30 gpurun_out/bench_tr1.log; exit 1; }
tail -1 gpurun_out/bench_tr1.log | cut -c1-200

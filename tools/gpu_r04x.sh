#!/bin/bash
# r04x: the multi-rank launcher and the N = 2 / 4 / 8 share paths on one card (gloo all-reduce,
# every rank on GPU 0: a functional rehearsal of the driver's scaling runs, not a scaling figure)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
for n in 2 4 8; do
  timeout -k 10 400 python bench.py --gpus $n --dist-backend gloo --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/r04x_g$n.json 2> gpurun_out/r04x_g$n.err || { echo "gpus $n failed"; tail -20 gpurun_out/r04x_g$n.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r04x_g$n.json').read().strip().splitlines()[-1]); print($n, d['value'], d['ms_per_step'], d['config'].get('lanes_per_gpu'), d['config'].get('parallelism'))"
done

#!/bin/bash
# r04m: the default bench line twice on one box (CPU baseline with the discarded warm-up run)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 500 python bench.py > gpurun_out/r04m_bench_$i.json 2> gpurun_out/r04m_bench_$i.err || { tail -20 gpurun_out/r04m_bench_$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r04m_bench_$i.json')); c=d['cpu_baseline']; print(d['value'], d['roofline']['frac'], d['roofline']['traffic'], c['value'], c['warmup_run'], c['end_to_end_runs'], c['spread'])"
done

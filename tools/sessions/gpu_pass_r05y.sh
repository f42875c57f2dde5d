# r05y: the 40 000-sample rollout at other lane x step splits (bench --max-lanes: 8192 x 5 default, 10240 x 4,
# 20480 x 2, 40960 x 1) -- how much of the rollout is per-step fixed cost; information for the lane-plan model
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
for r in 1 2; do for m in 8192 10240 20480 40960; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --max-lanes $m > gpurun_out/r05y_lanes_$m.json 2>/dev/null || { echo "max-lanes $m failed"; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/r05y_lanes_$m.json')); print('round $r max-lanes $m', d['value'], d['ms_per_step'], d['config'].get('lanes_per_gpu'), d['config'].get('sync_steps'), d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done; done

#!/bin/bash
# r03f: the -m gpu suite on the build with batched stream-K combine loads and the NPG column
# reduces 8 loads deep; old/new A/B (tools/so_ab.sh) of the N = 8 / 4 / 2 per-rank shares and
# of the NPG update; the default bench line on the new build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r03f.log 2>&1 || { tail -30 gpurun_out/pytest_r03f.log; exit 1; }
tail -1 gpurun_out/pytest_r03f.log
bash tools/so_ab.sh 1 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --total-samples 5000 --expert-rows 6250 > gpurun_out/r03f_share5k_ab.txt 2>&1 || { tail -20 gpurun_out/r03f_share5k_ab.txt; exit 1; }
bash tools/so_ab.sh 1 python tools/npg_time.py > gpurun_out/r03f_npg_ab.txt 2>&1 || { tail -20 gpurun_out/r03f_npg_ab.txt; exit 1; }
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03f_bench.json 2> gpurun_out/r03f_bench.err || { tail -20 gpurun_out/r03f_bench.err; exit 1; }
for f in share5k; do echo "== $f"; grep -E '^==|"value"' gpurun_out/r03f_${f}_ab.txt | grep -v amdgpu | sed -E 's/.*"value": ([0-9.]+).*"ms_per_step": ([0-9.]+).*/\1 \2/'; done
grep -v amdgpu.ids gpurun_out/r03f_npg_ab.txt | cut -c1-160
cut -c1-200 gpurun_out/r03f_bench.json

#!/bin/bash
# r04a: the -m gpu suite + smoke on the build with the batched stream-K combine (and the round-4
# sampler fixes); old/new A/B of the N = 8 / 4 per-rank shares; the timed-region rocprofv3 kernel
# trace of the default bench; the PMC traffic passes (FETCH_SIZE, WRITE_SIZE) of this build; the
# NPG update time; the default bench line with the CPU baseline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; L=$R/amp_extensions_amd
cd "$R" && mkdir -p gpurun_out
cp $L/libamx_hip_new.so $L/libamx_hip.so
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r04a.log 2>&1; rc=$?; [ $rc -le 1 ] || { tail -40 gpurun_out/pytest_r04a.log; exit 1; }; grep -E "^FAILED" gpurun_out/pytest_r04a.log
tail -1 gpurun_out/pytest_r04a.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04a.log 2>&1 || { tail -20 gpurun_out/smoke_r04a.log; exit 1; }
tail -1 gpurun_out/smoke_r04a.log
bash tools/so_ab.sh 2 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --total-samples 5000 --expert-rows 6250 > gpurun_out/r04a_share5k_ab.txt 2>&1 || { tail -20 gpurun_out/r04a_share5k_ab.txt; exit 1; }
bash tools/so_ab.sh 1 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --total-samples 10000 --expert-rows 12500 > gpurun_out/r04a_share10k_ab.txt 2>&1 || { tail -20 gpurun_out/r04a_share10k_ab.txt; exit 1; }
cp $L/libamx_hip_new.so $L/libamx_hip.so
timeout -k 10 200 python tools/npg_time.py > gpurun_out/r04a_npg_time.txt 2>&1 || { tail -20 gpurun_out/r04a_npg_time.txt; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r04a" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 > "$R/gpurun_out/prof_r04a.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_r04a.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r04a_5k" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --total-samples 5000 --expert-rows 6250 --steps 10 --warmup 2 > "$R/gpurun_out/prof_r04a_5k.log" 2>&1 || { echo "rocprof 5k failed"; tail -5 "$R/gpurun_out/prof_r04a_5k.log"; exit 1; }
cd "$R"
bash tools/pmc_traffic.sh r04a f16x3 > gpurun_out/r04a_pmc.txt 2>&1 || { tail -20 gpurun_out/r04a_pmc.txt; exit 1; }
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || { tail -20 gpurun_out/r04a_bench.err; exit 1; }
for f in share5k share10k; do echo "== $f"; grep -E '^==|"value"' gpurun_out/r04a_${f}_ab.txt | grep -v amdgpu | sed -E 's/.*"value": ([0-9.]+).*"ms_per_step": ([0-9.]+).*/\1 \2/'; done
tail -3 gpurun_out/r04a_npg_time.txt | cut -c1-200
tail -1 gpurun_out/r04a_pmc.txt
cut -c1-300 gpurun_out/r04a_bench.json

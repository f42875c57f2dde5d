# r05d: full -m gpu suite on the pruned default build, smoke, the PMC traffic record of the
# rebuilt GEMM source, the default bench line, the one-card gloo rehearsal of --gpus 2 (dist_diag
# fields), and the N = 8 share's kernel timeline with graph replay on and off (k_assemble).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; L=$R/amp_extensions_amd; cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r05d_pytest.log 2>&1; rc=$?
[ $rc -le 1 ] || { tail -40 gpurun_out/r05d_pytest.log; exit 1; }
grep -E "^FAILED|^ERROR" gpurun_out/r05d_pytest.log; tail -1 gpurun_out/r05d_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05d_smoke.log 2>&1 || { tail -20 gpurun_out/r05d_smoke.log; exit 1; }
tail -1 gpurun_out/r05d_smoke.log
bash tools/pmc_traffic.sh r05d f16x3 > gpurun_out/r05d_pmc.txt 2>&1 || { tail -20 gpurun_out/r05d_pmc.txt; exit 1; }
tail -1 gpurun_out/r05d_pmc.txt
cp gpurun_out/gemm_traffic_f16x3.json $L/data/gemm_traffic_f16x3.json
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r05d_bench.json 2> gpurun_out/r05d_bench.err || { tail -20 gpurun_out/r05d_bench.err; exit 1; }
cut -c1-220 gpurun_out/r05d_bench.json
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r05d_gloo2.json 2> gpurun_out/r05d_gloo2.err || { tail -20 gpurun_out/r05d_gloo2.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r05d_gloo2.json').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d.get('dist_diag')))"
cd /tmp && export TMPDIR=/tmp
for g in on off; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r05d_5k_$g" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --total-samples 5000 --expert-rows 6250 --steps 20 --warmup 5 --graph $g > "$R/gpurun_out/prof_r05d_5k_$g.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_r05d_5k_$g.log"; exit 1; }
done
cd "$R"
for g in on off; do python tools/trace_timeline.py gpurun_out/prof_r05d_5k_$g/run_kernel_trace.csv > gpurun_out/r05d_timeline_5k_$g.txt; tail -12 gpurun_out/r05d_timeline_5k_$g.txt; done
bash tools/ab_bench.sh "t0 t1 f1" 3 --steps 20 --warmup 5 | tee gpurun_out/r05d_trans_ab_8k.txt
bash tools/ab_bench.sh "t0 t1 f1" 3 --total-samples 5000 --expert-rows 6250 --steps 50 --warmup 10 | tee gpurun_out/r05d_trans_ab_5k.txt

# r05i: the one-launch forward (amx_forward_h3): bit-identity vs the per-layer launches + the forward /
# share / parity tests, then same-box A/B on bench lines (N = 1 default, N = 8 share): per-layer
# launches vs fused (FW_CT 1, shipped) vs fused FW_CT 0 vs fused FW_DRAIN 0 (nd); and a rocprof kernel trace of the fused N = 1 bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fwd.py tests/test_gpu_h3.py tests/test_gpu_share_shapes.py tests/test_gpu_parity.py > gpurun_out/r05i_pytest.log 2>&1 || { tail -60 gpurun_out/r05i_pytest.log; exit 1; }
tail -3 gpurun_out/r05i_pytest.log
cp amp_extensions_amd/libamx_hip.so /tmp/libamx_orig.so
line() { python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_us"], d["roofline"]["frac"])'; }
for r in 1 2; do for v in layers:ct1 fused:ct1 fused:ct0 fused:nd; do
  f=${v%%:*}; t=${v##*:}
  cp amp_extensions_amd/libamx_hip_$t.so amp_extensions_amd/libamx_hip.so
  out=$(timeout -k 10 200 python bench.py --no-cpu-baseline --forward $f 2>/dev/null | tail -1) || { echo "bench $v failed"; cp /tmp/libamx_orig.so amp_extensions_amd/libamx_hip.so; exit 1; }
  echo "n1 $f-$t r$r $(echo "$out" | line)"
  out=$(timeout -k 10 200 python bench.py --no-cpu-baseline --forward $f --total-samples 5000 --expert-rows 6250 --steps 50 --warmup 10 2>/dev/null | tail -1) || { echo "share $v failed"; cp /tmp/libamx_orig.so amp_extensions_amd/libamx_hip.so; exit 1; }
  echo "share $f-$t r$r $(echo "$out" | line)"
done; done | tee gpurun_out/r05i_ab.txt
cp /tmp/libamx_orig.so amp_extensions_amd/libamx_hip.so
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r05i" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --steps 10 --warmup 3 > "$R/gpurun_out/prof_r05i.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_r05i.log"; exit 1; }
cd "$R" && head -12 gpurun_out/prof_r05i/run_kernel_stats.csv | cut -c1-200

# r05m: the one-launch forward with one barrier per boundary, LDS-staged bias, no epilogue drain (base) vs
# the same with the drain (dr) vs the per-layer launches at the N = 8 share; tests first; stamps
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fwd.py tests/test_gpu_share_shapes.py tests/test_gpu_parity.py tests/test_gpu_h3.py > gpurun_out/r05m_pytest.log 2>&1 || { tail -40 gpurun_out/r05m_pytest.log; exit 1; }
tail -2 gpurun_out/r05m_pytest.log
cp amp_extensions_amd/libamx_hip.so /tmp/libamx_orig.so
cp amp_extensions_amd/libamx_hip.so amp_extensions_amd/libamx_hip_base.so
cp amp_extensions_amd/libamx_hip_fwt.so amp_extensions_amd/libamx_hip.so
timeout -k 10 200 python tools/fwd_trace.py 5120 > gpurun_out/r05m_fwd_trace.txt 2>&1; rc=$?
cp /tmp/libamx_orig.so amp_extensions_amd/libamx_hip.so
cat gpurun_out/r05m_fwd_trace.txt; [ $rc -eq 0 ] || exit 1
line() { python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_us"], d["roofline"]["frac"])'; }
for r in 1 2 3; do for v in layers:base fused:base fused:dr; do
  f=${v%%:*}; t=${v##*:}
  cp amp_extensions_amd/libamx_hip_$t.so amp_extensions_amd/libamx_hip.so
  out=$(timeout -k 10 200 python bench.py --no-cpu-baseline --forward $f --total-samples 5000 --expert-rows 6250 --steps 50 --warmup 10 2>/dev/null | tail -1) || { echo "share $v failed"; cp /tmp/libamx_orig.so amp_extensions_amd/libamx_hip.so; exit 1; }
  echo "share $f-$t r$r $(echo "$out" | line)"
done; done | tee gpurun_out/r05m_ab.txt
cp /tmp/libamx_orig.so amp_extensions_amd/libamx_hip.so

# r05s: the one-launch forward streaming half of each slice through LDS (fs) vs the whole-slice epilogue (fn) vs the
# per-layer launches (default library) at the N = 8 / N = 4 shares; its tests on the experimental build; stamps (fst)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
cp amp_extensions_amd/libamx_hip.so /tmp/libamx_orig.so
cp amp_extensions_amd/libamx_hip.so amp_extensions_amd/libamx_hip_base.so
restore() { cp /tmp/libamx_orig.so amp_extensions_amd/libamx_hip.so; }
cp amp_extensions_amd/libamx_hip_fs.so amp_extensions_amd/libamx_hip.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fwd.py tests/test_gpu_share_shapes.py > gpurun_out/r05s_pytest.log 2>&1 || { restore; tail -40 gpurun_out/r05s_pytest.log; exit 1; }
tail -1 gpurun_out/r05s_pytest.log
cp amp_extensions_amd/libamx_hip_fst.so amp_extensions_amd/libamx_hip.so
AMX_FORWARD=fused timeout -k 10 200 python tools/fwd_trace.py 5120 > gpurun_out/r05s_fwd_trace.txt 2>&1; rc=$?
restore; grep -v amdgpu.ids gpurun_out/r05s_fwd_trace.txt; [ $rc -eq 0 ] || exit 1
line() { python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_us"])'; }
for r in 1 2 3; do for v in layers:base fused:fs fused:fn; do
  f=${v%%:*}; t=${v##*:}
  cp amp_extensions_amd/libamx_hip_$t.so amp_extensions_amd/libamx_hip.so
  out=$(timeout -k 10 200 python bench.py --no-cpu-baseline --forward $f --total-samples 5000 --expert-rows 6250 --steps 50 --warmup 10 2>/dev/null | tail -1) || { echo "share $v failed"; restore; exit 1; }
  echo "share8 $f-$t r$r $(echo "$out" | line)"
  out=$(timeout -k 10 200 python bench.py --no-cpu-baseline --forward $f --total-samples 10000 --expert-rows 12500 --steps 30 --warmup 5 2>/dev/null | tail -1) || { echo "share4 $v failed"; restore; exit 1; }
  echo "share4 $f-$t r$r $(echo "$out" | line)"
done; done | tee gpurun_out/r05s_ab.txt
restore

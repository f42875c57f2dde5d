# r05k: the one-launch forward with the fragment-ordered weight image: tests, per-layer stamps, A/B vs
# the per-layer launches on bench lines (N = 1, N = 8 share), L1/TA counters of the fused forward
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fwd.py tests/test_gpu_share_shapes.py tests/test_gpu_parity.py > gpurun_out/r05k_pytest.log 2>&1 || { tail -40 gpurun_out/r05k_pytest.log; exit 1; }
tail -2 gpurun_out/r05k_pytest.log
cp amp_extensions_amd/libamx_hip.so /tmp/libamx_orig.so
cp amp_extensions_amd/libamx_hip_fwt.so amp_extensions_amd/libamx_hip.so
timeout -k 10 200 python tools/fwd_trace.py 5120 8192 > gpurun_out/r05k_fwd_trace.txt 2>&1; rc=$?
cp /tmp/libamx_orig.so amp_extensions_amd/libamx_hip.so
cat gpurun_out/r05k_fwd_trace.txt; [ $rc -eq 0 ] || exit 1
line() { python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_us"], d["roofline"]["frac"])'; }
for r in 1 2; do for f in layers fused; do
  out=$(timeout -k 10 200 python bench.py --no-cpu-baseline --forward $f 2>/dev/null | tail -1) || { echo "bench $f failed"; exit 1; }
  echo "n1 $f r$r $(echo "$out" | line)"
  out=$(timeout -k 10 200 python bench.py --no-cpu-baseline --forward $f --total-samples 5000 --expert-rows 6250 --steps 50 --warmup 10 2>/dev/null | tail -1) || { echo "share $f failed"; exit 1; }
  echo "share $f r$r $(echo "$out" | line)"
done; done | tee gpurun_out/r05k_ab.txt
cd /tmp && export TMPDIR=/tmp
P3="TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCP_PENDING_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES TCP_CACHE_MISS TCP_PERF_SEL_TOTAL_READ TCC_HIT TCC_MISS GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $P3 -d "$R/gpurun_out/fwdpmc_k_3" -o run --output-format csv -- python "$R/tools/fwd_pmc.py" run fused 5120 20 > "$R/gpurun_out/fwdpmc_k_3.log" 2>&1 || { echo "pmc failed"; exit 1; }
cd "$R" && python tools/fwd_pmc.py parse gpurun_out/fwdpmc_k_3

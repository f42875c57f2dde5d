# r05p: the policy's noise computed under its staging loads: policy / sampler / share tests, phase stamps,
# same-box share + N = 1 A/B against the previous amx_step build (polold), NPG timing
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_policy_shapes.py tests/test_gpu_share_shapes.py tests/test_gpu_sampler.py tests/test_gpu_configs.py > gpurun_out/r05p_pytest.log 2>&1 || { tail -40 gpurun_out/r05p_pytest.log; exit 1; }
tail -1 gpurun_out/r05p_pytest.log
cp amp_extensions_amd/libamx_hip.so /tmp/libamx_orig.so
cp amp_extensions_amd/libamx_hip.so amp_extensions_amd/libamx_hip_polnew.so
cp amp_extensions_amd/libamx_hip_polt.so amp_extensions_amd/libamx_hip.so
timeout -k 10 200 python tools/policy_trace.py 5120 8192 > gpurun_out/r05p_policy_trace.txt 2>&1; rc=$?
cp /tmp/libamx_orig.so amp_extensions_amd/libamx_hip.so
grep -v amdgpu.ids gpurun_out/r05p_policy_trace.txt; [ $rc -eq 0 ] || exit 1
line() { python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for r in 1 2 3; do for t in polold polnew; do
  cp amp_extensions_amd/libamx_hip_$t.so amp_extensions_amd/libamx_hip.so
  out=$(timeout -k 10 200 python bench.py --no-cpu-baseline --total-samples 5000 --expert-rows 6250 --steps 50 --warmup 10 2>/dev/null | tail -1) || { echo "share $t failed"; cp /tmp/libamx_orig.so amp_extensions_amd/libamx_hip.so; exit 1; }
  echo "share $t r$r $(echo "$out" | line)"
  out=$(timeout -k 10 200 python bench.py --no-cpu-baseline 2>/dev/null | tail -1) || { echo "n1 $t failed"; cp /tmp/libamx_orig.so amp_extensions_amd/libamx_hip.so; exit 1; }
  echo "n1 $t r$r $(echo "$out" | line)"
done; done | tee gpurun_out/r05p_ab.txt
cp /tmp/libamx_orig.so amp_extensions_amd/libamx_hip.so
timeout -k 10 300 python tools/npg_time.py > gpurun_out/r05p_npg_time.txt 2>&1 || { tail -5 gpurun_out/r05p_npg_time.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r05p_npg_time.txt

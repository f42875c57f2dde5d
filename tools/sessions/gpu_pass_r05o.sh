# r05o: policy kernel phase stamps (POL_TRACE build) at 5120 / 8192 lanes; NPG update time with consecutive updates
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
cp amp_extensions_amd/libamx_hip.so /tmp/libamx_orig.so
cp amp_extensions_amd/libamx_hip_polt.so amp_extensions_amd/libamx_hip.so
timeout -k 10 200 python tools/policy_trace.py 5120 8192 > gpurun_out/r05o_policy_trace.txt 2>&1; rc=$?
cp /tmp/libamx_orig.so amp_extensions_amd/libamx_hip.so
grep -v amdgpu.ids gpurun_out/r05o_policy_trace.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/npg_time.py > gpurun_out/r05o_npg_time.txt 2>&1 || { tail -5 gpurun_out/r05o_npg_time.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r05o_npg_time.txt

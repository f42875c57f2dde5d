# r05h: per-phase stamps of the f16x3 forward's launches (H3_TRACE build) at the N = 8 share and at N = 1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
cp amp_extensions_amd/libamx_hip.so /tmp/libamx_orig.so
cp amp_extensions_amd/libamx_hip_h3t.so amp_extensions_amd/libamx_hip.so
timeout -k 10 300 python tools/h3_trace.py 5120 8192 > gpurun_out/r05h_h3_trace.txt 2>&1; rc=$?
cp /tmp/libamx_orig.so amp_extensions_amd/libamx_hip.so
cat gpurun_out/r05h_h3_trace.txt; exit $rc

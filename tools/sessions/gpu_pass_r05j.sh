# r05j: where the one-launch forward's time goes: per-layer phase stamps (FW_TRACE builds, FW_CT 1 / 0)
# at 5120 / 8192 lanes, then counter passes fused vs per-layer at 5120 lanes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
cp amp_extensions_amd/libamx_hip.so /tmp/libamx_orig.so
for t in fwt fwt0; do
  cp amp_extensions_amd/libamx_hip_$t.so amp_extensions_amd/libamx_hip.so
  echo "== $t" >> gpurun_out/r05j_fwd_trace.txt
  timeout -k 10 200 python tools/fwd_trace.py 5120 8192 >> gpurun_out/r05j_fwd_trace.txt 2>&1 || { cp /tmp/libamx_orig.so amp_extensions_amd/libamx_hip.so; cat gpurun_out/r05j_fwd_trace.txt; exit 1; }
done
cp /tmp/libamx_orig.so amp_extensions_amd/libamx_hip.so
cat gpurun_out/r05j_fwd_trace.txt
bash tools/fwd_pmc.sh 5120 > gpurun_out/r05j_fwd_pmc.txt 2>&1; rc=$?
cat gpurun_out/r05j_fwd_pmc.txt; exit $rc

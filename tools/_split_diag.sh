mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for t in base nl ns nlns; do
  cp amp_extensions_amd/libamx_hip_$t.so amp_extensions_amd/libamx_hip.so
  OUT_TILES=1 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/v_$t -o run -- python3 -u tools/out_ab.py 8192 > gpurun_out/v_$t.txt 2>&1 || exit 1
done
cp amp_extensions_amd/libamx_hip_base.so amp_extensions_amd/libamx_hip.so

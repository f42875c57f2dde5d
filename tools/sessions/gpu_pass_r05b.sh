set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
cp amp_extensions_amd/libamx_hip_o160.so amp_extensions_amd/libamx_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_share_shapes.py tests/test_gpu_out_ring.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05b_pytest.log 2>&1 || { tail -40 gpurun_out/r05b_pytest.log; exit 1; }
tail -1 gpurun_out/r05b_pytest.log
cp amp_extensions_amd/libamx_hip_base.so amp_extensions_amd/libamx_hip.so
bash tools/ab_bench.sh "base o160" 3 --total-samples 5000 --expert-rows 6250 --steps 50 --warmup 10 | tee gpurun_out/r05b_ab.txt

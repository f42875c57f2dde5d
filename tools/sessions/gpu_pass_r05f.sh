# r05f: K-loop staging schedule A/B: b0 round-4 (fenced barrier, pieces behind every m-block),
# b1 unfenced K-loop barrier, b2 b1 + pieces front-loaded into the first half of the m-blocks,
# b3 fenced barrier + front-loaded pieces; GEMM / share tests on b2 first.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
cp amp_extensions_amd/libamx_hip.so /tmp/libamx_orig.so
cp amp_extensions_amd/libamx_hip_b2.so amp_extensions_amd/libamx_hip.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_h3.py tests/test_gpu_parity.py tests/test_gpu_share_shapes.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05f_pytest.log 2>&1 || { tail -40 gpurun_out/r05f_pytest.log; exit 1; }
tail -1 gpurun_out/r05f_pytest.log
cp /tmp/libamx_orig.so amp_extensions_amd/libamx_hip.so
bash tools/ab_bench.sh "b0 b1 b2 b3" 3 --steps 20 --warmup 5 | tee gpurun_out/r05f_ab_8k.txt
bash tools/ab_bench.sh "b0 b1 b2 b3" 3 --total-samples 5000 --expert-rows 6250 --steps 50 --warmup 10 | tee gpurun_out/r05f_ab_5k.txt

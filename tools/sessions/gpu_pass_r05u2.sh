# r05u2: the RFF column-partial sums (k_feature_message / k_sum_partials) on 16-column blocks with 64 row runs per column
# (mnew) vs 64-column blocks with 16 runs (mold): relabel / edges / multirank / configs tests on mnew, the message's
# launch time, N = 1 and share bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_relabel_fused.py tests/test_gpu_edges.py tests/test_gpu_multirank.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_share_shapes.py > gpurun_out/r05u2_pytest.log 2>&1 || { tail -40 gpurun_out/r05u2_pytest.log; exit 1; }
tail -1 gpurun_out/r05u2_pytest.log
timeout -k 10 300 bash tools/lib_ab.sh "mold mnew" 2 python tools/msg_time.py > gpurun_out/r05u2_msg.txt 2>&1 || { tail -20 gpurun_out/r05u2_msg.txt; exit 1; }
grep -E "==|feature" gpurun_out/r05u2_msg.txt
for r in 1 2 3; do for t in mold mnew; do
  cp amp_extensions_amd/libamx_hip_$t.so amp_extensions_amd/libamx_hip.so
  a=$(timeout -k 10 200 python bench.py --no-cpu-baseline --total-samples 5000 --expert-rows 6250 --steps 50 --warmup 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
  b=$(timeout -k 10 200 python bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
  echo "round $r $t share $a n1 $b"
done; done
cp amp_extensions_amd/libamx_hip_mnew.so amp_extensions_amd/libamx_hip.so

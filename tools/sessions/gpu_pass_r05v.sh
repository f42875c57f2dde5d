# r05v: the policy MLP on one wave (three layers, no workgroup barriers between them) with the noise drawn by the
# other three waves in parallel (pnew) vs the four-wave layers + combine passes (pold): policy / step-act / sampler /
# parity tests on pnew, kernel_micro A/B, share and N = 1 bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_policy_shapes.py tests/test_gpu_step_reset.py tests/test_gpu_parity.py tests/test_gpu_sampler.py tests/test_gpu_simenv_dropin.py tests/test_gpu_share_shapes.py tests/test_gpu_configs.py > gpurun_out/r05v_pytest.log 2>&1 || { tail -40 gpurun_out/r05v_pytest.log; exit 1; }
tail -1 gpurun_out/r05v_pytest.log
for L in 8192 5120; do
  timeout -k 10 400 bash tools/lib_ab.sh "pold pnew" 2 python tools/kernel_micro.py $L > gpurun_out/r05v_micro_$L.txt 2>&1 || { tail -20 gpurun_out/r05v_micro_$L.txt; exit 1; }
  grep -E "==|policy" gpurun_out/r05v_micro_$L.txt
done
for r in 1 2 3; do for t in pold pnew; do
  cp amp_extensions_amd/libamx_hip_$t.so amp_extensions_amd/libamx_hip.so
  a=$(timeout -k 10 200 python bench.py --no-cpu-baseline --total-samples 5000 --expert-rows 6250 --steps 50 --warmup 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
  b=$(timeout -k 10 200 python bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
  echo "round $r $t share $a n1 $b"
done; done
cp amp_extensions_amd/libamx_hip_pnew.so amp_extensions_amd/libamx_hip.so

# r05u4: k_assemble with every load of the row issued before the arithmetic (anew) vs one round trip per 64 columns
# (aold): assembly / parity / step tests on anew, kernel_micro A/B, N = 1 and share bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_step_reset.py tests/test_gpu_step_act.py tests/test_gpu_h3.py tests/test_gpu_share_shapes.py > gpurun_out/r05u4_pytest.log 2>&1 || { tail -40 gpurun_out/r05u4_pytest.log; exit 1; }
tail -1 gpurun_out/r05u4_pytest.log
for L in 8192 5120; do
  timeout -k 10 400 bash tools/lib_ab.sh "aold anew" 2 python tools/kernel_micro.py $L > gpurun_out/r05u4_micro_$L.txt 2>&1 || { tail -20 gpurun_out/r05u4_micro_$L.txt; exit 1; }
  grep -E "==|assemble" gpurun_out/r05u4_micro_$L.txt
done
for r in 1 2 3; do for t in aold anew; do
  cp amp_extensions_amd/libamx_hip_$t.so amp_extensions_amd/libamx_hip.so
  a=$(timeout -k 10 200 python bench.py --no-cpu-baseline --total-samples 5000 --expert-rows 6250 --steps 50 --warmup 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
  b=$(timeout -k 10 200 python bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
  echo "round $r $t share $a n1 $b"
done; done
cp amp_extensions_amd/libamx_hip_anew.so amp_extensions_amd/libamx_hip.so

# r05u5: the relabel rollout waves with two row batches each (rnew) vs one (rold)
# configs / multirank tests on rnew, the launch time at the N = 1 and N = 8 shapes (bit hash), N = 1 bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_relabel_fused.py tests/test_gpu_configs.py tests/test_gpu_multirank.py tests/test_gpu_edges.py > gpurun_out/r05u5_pytest.log 2>&1 || { tail -40 gpurun_out/r05u5_pytest.log; exit 1; }
tail -1 gpurun_out/r05u5_pytest.log
timeout -k 10 300 bash tools/lib_ab.sh "rold rnew" 2 python tools/relabel_time2.py > gpurun_out/r05u5_relabel.txt 2>&1 || { tail -20 gpurun_out/r05u5_relabel.txt; exit 1; }
grep -E "==|relabel" gpurun_out/r05u5_relabel.txt
for r in 1 2 3; do for t in rold rnew; do
  cp amp_extensions_amd/libamx_hip_$t.so amp_extensions_amd/libamx_hip.so
  b=$(timeout -k 10 200 python bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
  echo "round $r $t n1 $b"
done; done
cp amp_extensions_amd/libamx_hip_rnew.so amp_extensions_amd/libamx_hip.so

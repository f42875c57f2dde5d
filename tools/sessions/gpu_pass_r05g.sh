# r05g: NPG pass LDS strides 2 mod 4 (n1) vs round 4's 4 mod 8 (n0): NPG tests on n1, then the
# update time of each (tools/npg_time.py, alternating), and n1's kernel timeline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_npg.py tests/test_gpu_gae.py > gpurun_out/r05g_pytest.log 2>&1 || { tail -40 gpurun_out/r05g_pytest.log; exit 1; }
tail -1 gpurun_out/r05g_pytest.log
cp amp_extensions_amd/libamx_hip.so /tmp/libamx_orig.so
for r in 1 2 3; do for t in n0 n1; do
  cp amp_extensions_amd/libamx_hip_$t.so amp_extensions_amd/libamx_hip.so
  echo "$t r$r $(timeout -k 10 200 python tools/npg_time.py 2>/dev/null | grep 'device NPG' | cut -c1-120)"
done; done | tee gpurun_out/r05g_npg_ab.txt
cp /tmp/libamx_orig.so amp_extensions_amd/libamx_hip.so
cd /tmp && export TMPDIR=/tmp
for t in n0 n1; do
  cp "$R/amp_extensions_amd/libamx_hip_$t.so" "$R/amp_extensions_amd/libamx_hip.so"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r05g_$t" -o run --output-format csv -- python "$R/tools/npg_time.py" > "$R/gpurun_out/prof_r05g_$t.log" 2>&1 || { echo "rocprof failed"; exit 1; }
  cd "$R"; python tools/npg_timeline.py gpurun_out/prof_r05g_$t/run_kernel_trace.csv > gpurun_out/r05g_npg_timeline_$t.txt; echo "$t: $(grep 'k_npg<1' gpurun_out/r05g_npg_timeline_$t.txt | tail -1)"; cd /tmp
done
cp /tmp/libamx_orig.so "$R/amp_extensions_amd/libamx_hip.so"

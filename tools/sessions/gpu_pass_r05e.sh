# r05e: RFF features on 160-row tiles with 32-row column partials: GPU tests of the RFF / relabel /
# share paths, then a same-box A/B of the old tile choice (r0) and the 160-row tiles (r1) at N = 1
# and at the N = 8 share, with the RFF kernel's time from rocprof for each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_h3.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_share_shapes.py tests/test_gpu_edges.py tests/test_gpu_relabel_fused.py tests/test_gpu_cost_inputs.py tests/test_gpu_surfaces.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05e_pytest.log 2>&1 || { tail -40 gpurun_out/r05e_pytest.log; exit 1; }
tail -1 gpurun_out/r05e_pytest.log
bash tools/ab_bench.sh "r0 r1" 3 --steps 20 --warmup 5 | tee gpurun_out/r05e_rff_ab_8k.txt
bash tools/ab_bench.sh "r0 r1" 3 --total-samples 5000 --expert-rows 6250 --steps 50 --warmup 10 | tee gpurun_out/r05e_rff_ab_5k.txt
cd /tmp && export TMPDIR=/tmp
for t in r0 r1; do
  cp "$R/amp_extensions_amd/libamx_hip_$t.so" "$R/amp_extensions_amd/libamx_hip.so"
  for n in 40000 5000; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r05e_${t}_$n" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --total-samples $n --steps 20 --warmup 5 > "$R/gpurun_out/prof_r05e_${t}_$n.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_r05e_${t}_$n.log"; exit 1; }
    echo "$t $n: $(grep 'k_gemm_h3<2' $R/gpurun_out/prof_r05e_${t}_$n/run_kernel_stats.csv | cut -d, -f1-5)"
  done
done
cp "$R/amp_extensions_amd/libamx_hip_r1.so" "$R/amp_extensions_amd/libamx_hip.so"

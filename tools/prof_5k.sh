set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_5k" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --total-samples 5000 --steps 10 --warmup 2 > "$R/gpurun_out/prof_5k.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_5k.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_8k" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 > "$R/gpurun_out/prof_8k.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/prof_8k.log"; exit 1; }
echo done

#!/bin/bash
# PMC HBM-traffic passes for the ensemble GEMM (one counter per pass, no trace domains),
# then gpurun_out/gemm_traffic_<gemm>.json (copy to amp_extensions_amd/data/, where bench.py reads it).
# usage (on the GPU box): bash tools/pmc_traffic.sh [tag] [f16x3|bf16x6|f32]
set -o pipefail
TAG=${1:-r01}
GEMM=${2:-f16x3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -d "$R/gpurun_out/pmc_$C" -o run --output-format csv -- \
    python "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 --gemm $GEMM > "$R/gpurun_out/pmc_$C.log" 2>&1 \
    || { echo "rocprofv3 --pmc $C FAILED"; tail -20 "$R/gpurun_out/pmc_$C.log"; exit 1; }
done
cd "$R"
python tools/pmc_traffic.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE 8192 197 36 $GEMM > gpurun_out/gemm_traffic_$GEMM.json || exit 1
cp gpurun_out/pmc_FETCH_SIZE/run_counter_collection.csv "gpurun_out/${TAG}_pmc_fetch_size.csv"
cp gpurun_out/pmc_WRITE_SIZE/run_counter_collection.csv "gpurun_out/${TAG}_pmc_write_size.csv"
python -c "import json; d=json.load(open('gpurun_out/gemm_traffic_$GEMM.json')); print('traffic/launch', d['hbm_bytes_per_launch'], 'ratio', d['ratio'])"

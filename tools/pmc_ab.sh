#!/bin/bash
# SQ counter passes + kernel-trace durations of one f16x3 ensemble layer (tools/h3_pmc.py) for
# several prebuilt libraries (amp_extensions_amd/libamx_hip_<tag>.so), one rocprofv3 run per
# pass.  usage (GPU box): bash tools/pmc_ab.sh OUTTAG LAYER "tag1 tag2 ..."
set -o pipefail
OUT=$1; LAYER=$2; TAGS=$3
R=${GRAFT_REPO_ROOT:-$(pwd)}; L=$R/amp_extensions_amd
cp $L/libamx_hip.so /tmp/libamx_hip_restore.so
for v in $TAGS; do
  cp $L/libamx_hip_$v.so $L/libamx_hip.so
  bash "$R/tools/h3_pmc.sh" $LAYER > "$R/gpurun_out/${OUT}_$v.txt" 2>&1 || { cat "$R/gpurun_out/${OUT}_$v.txt"; cp /tmp/libamx_hip_restore.so $L/libamx_hip.so; exit 1; }
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${OUT}_kt_$v" -o run \
      --output-format csv -- python "$R/tools/h3_pmc.py" run $LAYER 40 > /dev/null 2>&1 ) || { echo "trace $v failed"; exit 1; }
  echo "== $v layer $LAYER" >> "$R/gpurun_out/${OUT}_$v.txt"
  grep k_gemm_h3 "$R/gpurun_out/${OUT}_kt_$v/run_kernel_stats.csv" | cut -d, -f1-8 >> "$R/gpurun_out/${OUT}_$v.txt"
  echo "== $v"; cat "$R/gpurun_out/${OUT}_$v.txt" | tail -25
done
cp /tmp/libamx_hip_restore.so $L/libamx_hip.so

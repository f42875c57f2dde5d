#!/bin/bash
# r04g: RFF pass A/B -- base (register epilogue, fast cos), cosf (register epilogue, OCML cosf),
# r3 (round 3's LDS-staged epilogue), r3f (staged epilogue + fast cos); diagnostics: nocos, nostore
# (RFF_EXP 1/2), nosplit (H3_EXP 2: A published unsplit), bare (both); interleaved processes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
for i in 1 2 3; do timeout -k 10 120 python tools/rff_ab.py base cosf r3 r3f nocos nostore nosplit bare || exit 1; done > gpurun_out/r04g_rff_ab.txt 2>&1 || { tail -20 gpurun_out/r04g_rff_ab.txt; exit 1; }
RFF_ROWS=5120 timeout -k 10 120 python tools/rff_ab.py base cosf r3 r3f nocos nostore nosplit bare >> gpurun_out/r04g_rff_ab.txt 2>&1 || { tail -20 gpurun_out/r04g_rff_ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04g_rff_ab.txt | cut -c1-200
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $C -d "$R/gpurun_out/pmc_rff_$C" -o run --output-format csv -- python "$R/tools/rff_ab.py" base > "$R/gpurun_out/pmc_rff_$C.log" 2>&1 || { echo "pmc $C failed"; tail -5 "$R/gpurun_out/pmc_rff_$C.log"; exit 1; }
done
cd "$R" && python tools/pmc_rff.py gpurun_out/pmc_rff_FETCH_SIZE gpurun_out/pmc_rff_WRITE_SIZE | tee gpurun_out/r04g_rff_pmc.txt

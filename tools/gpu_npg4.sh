#!/bin/bash
# NPG: parity tests, pass-variant timings, phase trace, update timing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
T=${1:-npg4}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_npg.py > $O/${T}_pytest.log 2>&1 || { tail -40 $O/${T}_pytest.log; exit 1; }
tail -2 $O/${T}_pytest.log
timeout -k 10 400 python -u tools/npg_phase.py run > $O/${T}_phase.txt 2>&1 || { cat $O/${T}_phase.txt; exit 1; }
cat $O/${T}_phase.txt
timeout -k 10 200 python -u tools/npg_phase.py trace > $O/${T}_trace.txt 2>&1 || { cat $O/${T}_trace.txt; exit 1; }
head -11 $O/${T}_trace.txt
timeout -k 10 240 python -u tools/npg_time.py 40960 197 36 16 > $O/${T}_time.txt 2>&1 || { cat $O/${T}_time.txt; exit 1; }
cat $O/${T}_time.txt

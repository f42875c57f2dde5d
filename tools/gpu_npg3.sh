#!/bin/bash
# NPG: parity tests, pass-variant timings, update timing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_npg.py > $O/npg3_pytest.log 2>&1 || { tail -40 $O/npg3_pytest.log; exit 1; }
tail -2 $O/npg3_pytest.log
timeout -k 10 400 python -u tools/npg_phase.py run > $O/npg_phase.txt 2>&1 || { cat $O/npg_phase.txt; exit 1; }
cat $O/npg_phase.txt
timeout -k 10 240 python -u tools/npg_time.py 40960 197 36 16 > $O/npg3_time.txt 2>&1 || { cat $O/npg3_time.txt; exit 1; }
cat $O/npg3_time.txt

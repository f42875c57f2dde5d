#!/bin/bash
# NPG pass kernel: parity tests, the update timing, and a kernel-trace profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_npg.py > $O/npg2_pytest.log 2>&1 || { tail -40 $O/npg2_pytest.log; exit 1; }
tail -3 $O/npg2_pytest.log
timeout -k 10 240 python -u tools/npg_time.py 40960 197 36 16 > $O/npg2_time.txt 2>&1 || { cat $O/npg2_time.txt; exit 1; }
cat $O/npg2_time.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_npg2 -o run --output-format csv -- python3 $R/tools/npg_time.py 40960 197 36 4 > $O/prof_npg2.log 2>&1 || { tail -20 $O/prof_npg2.log; exit 1; }
f=$(find $O/prof_npg2 -name 'run_kernel_stats.csv' | head -1)
head -8 "$f"

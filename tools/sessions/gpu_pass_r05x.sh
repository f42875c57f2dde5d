# r05x: the NPG CG tail in one launch (k_npg_cg_one: the column pass, a grid barrier, the vector step) vs the two
# launches (cg2 = NPG_CG_ONE 0): NPG / GAE tests on the one-launch build, npg_time A/B (update time, FVP, parameter
# hash: equal = bit-identical), training-mode bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_npg.py tests/test_gpu_gae.py > gpurun_out/r05x_pytest.log 2>&1 || { tail -40 gpurun_out/r05x_pytest.log; exit 1; }
tail -1 gpurun_out/r05x_pytest.log
timeout -k 10 500 bash tools/lib_ab.sh "cg2 cg1" 3 python tools/npg_time.py > gpurun_out/r05x_npg_ab.txt 2>&1 || { tail -20 gpurun_out/r05x_npg_ab.txt; exit 1; }
grep -E "==|consecutive|sha1|per update \(" gpurun_out/r05x_npg_ab.txt | cut -c1-160
timeout -k 10 600 bash tools/lib_ab.sh "cg2 cg1" 2 python bench.py --mode train --no-cpu-baseline > gpurun_out/r05x_train_ab.txt 2>&1 || { tail -20 gpurun_out/r05x_train_ab.txt; exit 1; }
grep -E "^==|^\{" gpurun_out/r05x_train_ab.txt | cut -c1-120

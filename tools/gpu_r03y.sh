set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03y; mkdir -p $out
bash tools/ab_env.sh DVIE_OP_LANES 0 1 ab_lanes || exit 1
bash tools/ab_env.sh DVIE_BRANCH_LANES 0 1 ab_branch || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_train.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" $out/pytest.log | head -20; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log

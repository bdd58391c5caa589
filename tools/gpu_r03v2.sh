set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03v2; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lanes.py -x -v --timeout 200 --timeout-method thread > $out/pytest_lanes.log 2>&1 || { echo "lane tests failed"; grep -E "FAIL|Error|assert" $out/pytest_lanes.log | head; exit 1; }
tail -1 $out/pytest_lanes.log
bash tools/ab_env.sh DVIE_BRANCH_LANES 0 1 ab_branch_eager || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log

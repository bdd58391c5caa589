set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r02b; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_dp.py -x -v -s --timeout 600 --timeout-method thread > $out/pytest_new.log 2>&1
rc=$?; tail -40 $out/pytest_new.log; exit $rc

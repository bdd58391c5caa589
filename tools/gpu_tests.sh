#!/bin/bash
# Run selected GPU test files on the box: bash tools/gpu_tests.sh <tag> <pytest args...>
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 1000 python -u -m pytest "$@" -x -v -s --timeout 600 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert" $out/pytest.log | tail -40; exit $rc

#!/bin/bash
# r04: the whole GPU test suite and smoke() on the current tree
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-r04t}; mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|assert" $out/pytest_gpu.log | head -20; tail -30 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log

#!/bin/bash
# warp forward: XCD-banded workgroup order A/B + warp parity
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-r04aa}; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k warp > $out/pytest_warp.log 2>&1 \
  || { tail -30 $out/pytest_warp.log; exit 1; }
tail -1 $out/pytest_warp.log
timeout -k 10 300 python -u tools/warp_ab.py DVIE_WARP_XCD 1 0 5 > $out/warp_xcd.txt 2>&1 || { tail -20 $out/warp_xcd.txt; exit 1; }
cat $out/warp_xcd.txt

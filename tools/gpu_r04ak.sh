#!/bin/bash
# fused head backward for both heads (DVIE_HEAD3_FUSED=2) vs rgb only (1), after the asm
# LDS-DMA change sped up head3_bwd_kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-r04ak}; mkdir -p $out
DVIE_HEAD3_FUSED=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_head3.py > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
bash tools/ab_env.sh DVIE_HEAD3_FUSED 2 1 ${1:-r04ak}/ab_head3 || exit 1

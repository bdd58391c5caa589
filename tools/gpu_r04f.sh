#!/bin/bash
# r04: fused-head / seg-encoder tests, then same-box A/B of the fusion defaults
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-r04f}; mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -s tests/test_gpu_head3.py tests/test_gpu_lanes.py \
  > $out/pytest.log 2>&1
rc=$?; grep -E "passed|failed|Error|assert|worst" $out/pytest.log | tail -20
[ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh DVIE_SEGENC_FWD 0 1 ${1:-r04f}/ab_segenc_fwd || exit 1
bash tools/ab_env.sh DVIE_HEAD3_FUSED 1 2 ${1:-r04f}/ab_head3 || exit 1
bash tools/ab_env.sh DVIE_HEAD3_FUSED 1 0 ${1:-r04f}/ab_head3_off || exit 1
